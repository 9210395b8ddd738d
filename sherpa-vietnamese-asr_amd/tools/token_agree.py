"""Token agreement of the precision modes on the benched hour (bench.py's workload).

    python sherpa-vietnamese-asr_amd/tools/token_agree.py [--modes bf16x6,bf16x3,bf16]
        [--methods greedy,beam8hw] [--audio-sec 3600] [--out gpurun_out/agree.json]

Decodes the same 121 planner chunks (bench.py make_chunks, same weights seed) once in the
exact-f32 mode and once per listed mode, and reports per mode and search method: chunks whose
token ids equal the fp32 decode, total tokens, and the token error rate (Levenshtein distance
over the fp32 tokens).  Diagnostic for DESIGN §6; bench.py's parity_mode carries the same
count for the mode it times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def edit_distance(a, b) -> int:
    a = list(a)
    b = list(b)
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="f16x3,bf16x6,bf16x3,bf16")
    ap.add_argument("--methods", default="greedy,beam8hw")
    ap.add_argument("--audio-sec", type=float, default=3600.0)
    ap.add_argument("--model", default="zipformer-68m")
    ap.add_argument("--out", default="")
    args = ap.parse_args()

    import torch
    import bench
    from zasr.binding import Recognizer
    from zasr.model import PRESETS, save_model_dir, synth_tokens, synth_weights

    cfg = PRESETS[args.model]()
    chunks = bench.make_chunks(args.audio_sec, bench.AUDIO_SEED)
    lens = [c.shape[0] for c in chunks]
    offs = np.cumsum([0] + lens[:-1]).tolist()
    mdir = os.path.join(tempfile.gettempdir(), f"zasr_agree_{os.getpid()}")
    save_model_dir(mdir, cfg, synth_weights(cfg, bench.WEIGHT_SEED), synth_tokens(cfg.vocab_size))
    d_wav = torch.from_numpy(np.concatenate(chunks)).to("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    hw = bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size)

    out = {"chunks": len(chunks), "audio_sec": args.audio_sec, "results": {}}
    for meth in args.methods.split(","):
        beam = 1 if meth == "greedy" else 8
        method = "greedy_search" if beam == 1 else "modified_beam_search"
        hot = hw if meth == "beam8hw" else None

        def decode(prec):
            rec = Recognizer(mdir, method, beam, hotwords=hot[0] if hot else None,
                             hotword_scores=hot[1] if hot else None, precision=prec)
            t0 = time.perf_counter()
            r = rec.decode_device(d_wav.data_ptr(), offs, lens, beam=beam, stream=stream)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            rec.close()
            return [x.token_ids.tolist() for x in r], el

        ref, _ = decode("fp32")
        nref = sum(len(t) for t in ref)
        for prec in args.modes.split(","):
            got, el = decode(prec)
            same = sum(a == b for a, b in zip(ref, got))
            errs = sum(edit_distance(a, b) if a != b else 0 for a, b in zip(ref, got))
            diff_chunks = [i for i, (a, b) in enumerate(zip(ref, got)) if a != b]
            rec = {"chunks_identical_to_fp32": f"{same}/{len(ref)}", "fp32_tokens": nref,
                   "token_errors": errs, "ter": round(errs / max(nref, 1), 6),
                   "differing_chunks": diff_chunks[:40]}
            out["results"][f"{meth}:{prec}"] = rec
            print(meth, prec, json.dumps(rec), flush=True)
    print(json.dumps(out))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
