"""Golden token ids of the BENCHED hour, decoded by the oracle (test infrastructure only).

bench.py's workload (make_chunks(3600, AUDIO_SEED): 121 planner chunks of seeded synthetic
speech; Zipformer-68M random-init weights, WEIGHT_SEED) decoded on the CPU by the oracle --
numpy fbank (oracle/fbank.py) -> torch fp32 encoder (oracle/zipformer.py) -> the reference's
`_ort_beam_search` restated (oracle/search.py, core/asr_engine.py:1023-1153, pinned by the
reference-generated search goldens) -- with

  * greedy (beam 1, BASELINE config 2's method), and
  * modified beam search, beam 8, with the reference's hotword.txt graph (config 3; the
    bench's `load_hotwords(DEFAULT_HOTWORDS)` phrases),

and every chunk's tokens and frames written to tests/golden/bench_hour_oracle.json together
with the chunk lengths and a checksum of the audio, so a GPU run can check that it decoded the
same hour.  bench.py's parity check and tests/test_gpu_hour.py compare the GPU decode with this
file; no GPU-side code reads the oracle.

With --set rover it decodes the same hour for BASELINE config 4 (bench.py --stage rover): the
ROVER pair's two models, Zipformer-30M (synth_weights, WEIGHT_SEED + 1) and Zipformer-68M
(synth_weights, WEIGHT_SEED), each modified beam search, beam 8, with hotword.txt, written to
tests/golden/bench_hour_oracle_rover.json (keys rover30m_beam8_hw / rover68m_beam8_hw).

Deterministic (seeded audio and weights, fp32 torch on the CPU with a fixed thread count per
worker).  Takes a few minutes on 8 cores:
    python tests/golden/make_bench_hour_golden.py [--workers 4 --threads 2] [--weights VARIANT]
    python tests/golden/make_bench_hour_golden.py --set rover
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

OUT = os.path.join(REPO, "tests", "golden", "bench_hour_oracle.json")


def golden_path(variant: str) -> str:
    """bench_hour_oracle.json for the default weights, bench_hour_oracle_<variant>.json else."""
    return OUT if variant == "greedy-calibrated" else OUT.replace(".json", f"_{variant}.json")
_W = {}


def audio_digest(chunks) -> str:
    h = hashlib.sha256()
    for c in chunks:
        h.update(np.ascontiguousarray(c, dtype=np.float32).tobytes())
    return h.hexdigest()[:32]


ROVER_MODELS = (("rover30m_beam8_hw", "zipformer-30m", 1), ("rover68m_beam8_hw", "zipformer-68m", 0))


def _init(threads, variant, which="hour"):
    import torch
    import bench
    from oracle.search import HotwordGraph
    from oracle.zipformer import ZipformerOracle
    from zasr.model import PRESETS, synth_weights, variant_weights
    torch.set_num_threads(threads)
    _W["which"] = which
    if which == "rover":  # bench_rover's pair: synth_weights(cfg, WEIGHT_SEED + 1 / + 0)
        _W["pair"] = []
        for key, name, ds in ROVER_MODELS:
            cfg = PRESETS[name]()
            phrases, scores = bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size)
            _W["pair"].append((key, ZipformerOracle(cfg, synth_weights(cfg, bench.WEIGHT_SEED + ds)),
                               HotwordGraph(phrases, scores)))
        return
    cfg = PRESETS["zipformer-68m"]()
    _W["orc"] = ZipformerOracle(cfg, variant_weights(cfg, bench.WEIGHT_SEED, variant))
    phrases, scores = bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size)
    _W["graph"] = HotwordGraph(phrases, scores)


def _run(job):
    from oracle.fbank import fbank
    from oracle.search import beam_search
    idx, chunk = job
    if _W["which"] == "rover":
        f = fbank(chunk)  # one fbank per chunk for both models, as the reference shares it
        out = {}
        for key, orc, graph in _W["pair"]:
            b = beam_search(orc.encoder(f), orc.decoder, orc.joiner, 8, graph)
            out[key] = [int(t) for t in b[0]]
            out[key + "_frames"] = [int(x) for x in b[1]]
            out["frames_" + key] = int(b[3])
        return idx, out
    orc = _W["orc"]
    enc = orc.encoder(fbank(chunk))
    g = beam_search(enc, orc.decoder, orc.joiner, 1)
    b = beam_search(enc, orc.decoder, orc.joiner, 8, _W["graph"])
    return idx, {"greedy": [int(t) for t in g[0]], "greedy_frames": [int(f) for f in g[1]],
                 "beam8_hw": [int(t) for t in b[0]], "beam8_hw_frames": [int(f) for f in b[1]],
                 "frames": int(g[3])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--limit", type=int, default=0, help="first N chunks only (a dry run)")
    ap.add_argument("--weights", default="greedy-calibrated",
                    help="zasr.model.WEIGHT_VARIANTS name (bench.py --weights)")
    ap.add_argument("--set", default="hour", choices=["hour", "rover"],
                    help="hour: 68M greedy + beam 8 (configs 2 / 3); rover: the config-4 pair")
    a = ap.parse_args()
    import multiprocessing as mp
    import bench
    chunks = bench.make_chunks(3600.0, bench.AUDIO_SEED)
    if a.limit:
        chunks = chunks[:a.limit]
    t0 = time.time()
    res = [None] * len(chunks)
    # longest chunks first so the pool drains evenly
    order = sorted(range(len(chunks)), key=lambda i: -chunks[i].shape[0])
    with mp.get_context("spawn").Pool(a.workers, initializer=_init,
                                      initargs=(a.threads, a.weights, a.set)) as pool:
        for n, (i, r) in enumerate(pool.imap_unordered(_run, [(i, chunks[i]) for i in order])):
            res[i] = r
            if n % 10 == 0:
                print(f"{n + 1}/{len(chunks)} chunks, {time.time() - t0:.0f} s", flush=True)
    if a.set == "rover":
        out = {"what": "oracle decode of bench.py --stage rover's hour (make_chunks(3600, "
                       "AUDIO_SEED)): zipformer-30m synth_weights(WEIGHT_SEED + 1) and zipformer-68m "
                       "synth_weights(WEIGHT_SEED), each beam 8 + hotword.txt",
               "generator": "tests/golden/make_bench_hour_golden.py --set rover",
               "audio_sha256_32": audio_digest(chunks),
               "chunk_samples": [int(c.shape[0]) for c in chunks]}
        for key, _, _ in ROVER_MODELS:
            out[key] = [r[key] for r in res]
            out[key + "_frames"] = [r[key + "_frames"] for r in res]
        out["tokens"] = {key: sum(len(r[key]) for r in res) for key, _, _ in ROVER_MODELS}
        path = OUT.replace(".json", "_rover.json")
        if a.limit:
            path = path.replace(".json", f"_first{a.limit}.json")
        with open(path, "w") as f:
            json.dump(out, f, separators=(",", ":"))
        print(f"wrote {path}: {out['tokens']} tokens, {time.time() - t0:.0f} s")
        return
    out = {
        "what": "oracle decode of bench.py's hour (make_chunks(3600, AUDIO_SEED), "
                f"zipformer-68m weights {a.weights} (WEIGHT_SEED)): greedy and beam 8 + hotword.txt",
        "weights": a.weights,
        "generator": "tests/golden/make_bench_hour_golden.py",
        "audio_sha256_32": audio_digest(chunks),
        "chunk_samples": [int(c.shape[0]) for c in chunks],
        "greedy": [r["greedy"] for r in res],
        "greedy_frames": [r["greedy_frames"] for r in res],
        "beam8_hw": [r["beam8_hw"] for r in res],
        "beam8_hw_frames": [r["beam8_hw_frames"] for r in res],
        "frames": [r["frames"] for r in res],
        "tokens": {"greedy": sum(len(r["greedy"]) for r in res),
                   "beam8_hw": sum(len(r["beam8_hw"]) for r in res)},
    }
    path = golden_path(a.weights)
    if a.limit:
        path = path.replace(".json", f"_first{a.limit}.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {path}: {out['tokens']} tokens, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
