"""Audit of the benched-hour chunks where the GPU's exact-f32-quality decodes (fp32, f16x3)
differ from the oracle's (tests/golden/bench_hour_oracle.json) -- test infrastructure, run in
the build container on the GPU's token lists (gpurun_out/hour_tokens_<prec>_<method>.json,
written by tests/test_gpu_hour.py):

    python tests/golden/make_bench_hour_audit.py [gpurun_out] [--weights VARIANT]

For every differing chunk it reruns the oracle (numpy fbank -> torch fp32 encoder -> the
reference's _ort_beam_search restated, core/asr_engine.py:1023-1153) and records:
  greedy    the first frame where the two decodes part, the oracle's log-prob margin there
            (its own token's log-prob minus the GPU's token's) -- a rounding-level tie sits far
            below the logits' scale; the search adds every candidate's log-prob to the
            hypothesis score in f32 (core/asr_engine.py:1099-1100), whose ulp at the scores of
            a 30 s chunk (|score| ~ 500-2000) is 3e-5-1.2e-4, so margins of that size are
            decided by rounding -- and whether the oracle itself changes its tokens when its
            encoder output is perturbed by ~1e-6 relative (two seeds; two f32 encoders, torch
            on the CPU and MFMA on the GPU, differ by ~3e-6 on these chunks);
  beam 8    the same perturbation test, and the frames where the oracle meets an EXACT f32 tie
            at the beam boundary (np.argpartition's introselect then decides which hypotheses
            stay, an order no other implementation reproduces).
With gpurun_out/hour_enc_fp32.npz (the GPU fp32 encoder output of the differing greedy
chunks, written by the GPU test) it also runs the oracle's search on the GPU's encoder output:
the GPU's tokens from it mean the two paths part only through the encoders' f32 rounding.
A chunk is allowed (tests/golden/bench_hour_audit.json "allowed_chunks") when the oracle
flips under the perturbation, or (greedy) its margin is below 1e-3, or (beam) it meets an
exact boundary tie, or the oracle's search on the GPU's encoder output gives the GPU's tokens.  The GPU tokens of each allowed chunk are stored with it, so the GPU test
also checks that the chunk still decodes to what was audited.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
for p in (REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

OUT = os.path.join(HERE, "bench_hour_audit.json")


def perturbed(enc, seed, rel=2.0 ** -20):
    u = np.random.default_rng(seed).integers(-1, 2, size=enc.shape).astype(np.float64)
    return (enc.astype(np.float64) * (1.0 + rel * u)).astype(np.float32)


def greedy_margin(enc, orc, ref_toks, ref_frames, got_toks, got_frames):
    from oracle.search import BLANK, CTX
    a = dict(zip(ref_frames, ref_toks))
    b = dict(zip(got_frames, got_toks))
    ctx = [BLANK] * CTX
    for t in range(enc.shape[0]):
        x, y = a.get(t, BLANK), b.get(t, BLANK)
        if x != y:
            dec = orc.decoder(np.array([ctx[-CTX:]], dtype=np.int64))
            lg = orc.joiner(enc[t:t + 1], dec).astype(np.float64)[0]
            lp = lg - lg.max() - np.log(np.exp(lg - lg.max()).sum())
            return t, float(lp[x] - lp[y])
        if x != BLANK:
            ctx.append(x)
    return -1, 0.0


def main():
    import torch

    import bench
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from oracle.zipformer import ZipformerOracle
    from zasr.model import PRESETS, variant_weights
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("src", nargs="?", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--weights", default="greedy-calibrated")
    ap.add_argument("--set", default="hour", choices=["hour", "rover"],
                    help="rover: the config-4 pair against bench_hour_oracle_rover.json")
    a = ap.parse_args()
    if a.set == "rover":
        return main_rover(a.src)
    src, variant = a.src, a.weights
    tag = "" if variant == "greedy-calibrated" else f"_{variant}"
    torch.set_num_threads(8)
    with open(os.path.join(HERE, f"bench_hour_oracle{tag}.json")) as f:
        gold = json.load(f)
    chunks = bench.make_chunks(3600.0, bench.AUDIO_SEED)
    cfg = PRESETS["zipformer-68m"]()
    orc = ZipformerOracle(cfg, variant_weights(cfg, bench.WEIGHT_SEED, variant))
    phrases, scores = bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size)
    graph = HotwordGraph(phrases, scores)
    out = {"what": "chunks of the benched hour where the GPU's fp32 / f16x3 decodes differ from "
                   "the oracle, each with the oracle-side evidence that it is an f32 tie",
           "generator": "tests/golden/make_bench_hour_audit.py"}
    for method, key, beam, g in (("greedy", "greedy", 1, None), ("beam8_hw", "beam8_hw", 8, graph)):
        got, frames = {}, {}
        for prec in ("fp32", "f16x3"):
            path = os.path.join(src, f"hour_tokens_{prec}_{method}{tag}.json")
            if os.path.exists(path):
                with open(path) as f:
                    d = json.load(f)
                # {"tokens": [...], "frames": [...]} (older runs: the token lists alone)
                got[prec] = d["tokens"] if isinstance(d, dict) else d
                if isinstance(d, dict):
                    frames[prec] = d["frames"]
        ref = gold[key]
        diff = sorted({i for toks in got.values() for i, (a, b) in enumerate(zip(toks, ref)) if a != b})
        entries, allowed = {}, []
        for i in diff:
            enc = orc.encoder(fbank(chunks[i]))
            flips = [beam_search(perturbed(enc, sd), orc.decoder, orc.joiner, beam, g)[0] != ref[i]
                     for sd in (1, 2)]
            e = {"gpu_tokens": {p: t[i] for p, t in got.items() if t[i] != ref[i]},
                 "oracle_tokens": len(ref[i]),
                 "oracle_flips_under_1e-6_perturbation": flips}
            ok = any(flips)
            if beam == 1:
                m = {}
                for p, t in got.items():
                    fr = frames.get(p)
                    if t[i] != ref[i] and fr is not None:
                        f0, mg = greedy_margin(enc, orc, ref[i], gold["greedy_frames"][i], t[i], fr[i])
                        m[p] = {"frame": f0, "margin": mg}
                        ok = ok or abs(mg) < 1e-3
                e["oracle_margin_at_first_difference"] = m
            else:
                ties = []
                beam_search(enc, orc.decoder, orc.joiner, beam, g, ties=ties)
                e["oracle_exact_boundary_tie_frames"] = ties[:32]
                ok = ok or bool(ties)
            encs = os.path.join(src, f"hour_enc_fp32_{method}{tag}.npz")
            if not os.path.exists(encs) and method == "greedy" and not tag:
                encs = os.path.join(src, "hour_enc_fp32.npz")  # round-5 first runs
            if os.path.exists(encs):
                with np.load(encs) as z:
                    if f"chunk{i}" in z.files:
                        eg = z[f"chunk{i}"]
                        n = min(len(eg), len(enc))
                        e["gpu_enc_max_rel_diff"] = float(np.max(np.abs(eg[:n] - enc[:n]) /
                                                                 np.maximum(1.0, np.abs(enc[:n]))))
                        # the oracle's own search on the GPU's encoder output: the GPU's tokens?
                        r = beam_search(eg, orc.decoder, orc.joiner, beam, g)[0]
                        e["oracle_search_on_gpu_enc_equals_gpu"] = any(
                            r == t[i] for t in got.values())
                        ok = ok or e["oracle_search_on_gpu_enc_equals_gpu"]
            e["allowed"] = ok
            if ok:
                allowed.append(i)
            entries[str(i)] = e
            print(method, i, json.dumps({k: v for k, v in e.items() if k != "gpu_tokens"}), flush=True)
        out[method] = {"differing_chunks": diff, "allowed_chunks": allowed, "chunks": entries}
    out["weights"] = variant
    path = OUT.replace(".json", f"{tag}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


def main_rover(src):
    """--set rover: the ROVER pair's beam 8 + hotword.txt decodes (tests/test_gpu_hour.py
    test_hour_rover_pair_matches_oracle token lists) against bench_hour_oracle_rover.json; the
    beam-8 evidence of main() (the oracle's perturbation flip, exact boundary ties)."""
    import torch

    import bench
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from oracle.zipformer import ZipformerOracle
    from zasr.model import PRESETS, synth_weights
    torch.set_num_threads(8)
    with open(os.path.join(HERE, "bench_hour_oracle_rover.json")) as f:
        gold = json.load(f)
    chunks = bench.make_chunks(3600.0, bench.AUDIO_SEED)
    out = {"what": "chunks of bench.py --stage rover's hour where the GPU's fp32 / f16x3 decodes "
                   "of either ROVER model differ from the oracle, each with the oracle-side "
                   "evidence that it is an f32 tie",
           "generator": "tests/golden/make_bench_hour_audit.py --set rover"}
    for model, name, ds in (("rover30m", "zipformer-30m", 1), ("rover68m", "zipformer-68m", 0)):
        key = f"{model}_beam8_hw"
        cfg = PRESETS[name]()
        orc = ZipformerOracle(cfg, synth_weights(cfg, bench.WEIGHT_SEED + ds))
        graph = HotwordGraph(*bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size))
        got = {}
        for prec in ("fp32", "f16x3"):
            path = os.path.join(src, f"hour_tokens_{prec}_{model}.json")
            if os.path.exists(path):
                with open(path) as f:
                    got[prec] = json.load(f)["tokens"]
        ref = gold[key]
        diff = sorted({i for toks in got.values() for i, (a, b) in enumerate(zip(toks, ref)) if a != b})
        entries, allowed = {}, []
        for i in diff:
            enc = orc.encoder(fbank(chunks[i]))
            flips = [beam_search(perturbed(enc, sd), orc.decoder, orc.joiner, 8, graph)[0] != ref[i]
                     for sd in (1, 2)]
            ties = []
            beam_search(enc, orc.decoder, orc.joiner, 8, graph, ties=ties)
            e = {"gpu_tokens": {p: t[i] for p, t in got.items() if t[i] != ref[i]},
                 "oracle_tokens": len(ref[i]),
                 "oracle_flips_under_1e-6_perturbation": flips,
                 "oracle_exact_boundary_tie_frames": ties[:32]}
            e["allowed"] = any(flips) or bool(ties)
            if e["allowed"]:
                allowed.append(i)
            entries[str(i)] = e
            print(key, i, json.dumps({k: v for k, v in e.items() if k != "gpu_tokens"}), flush=True)
        out[key] = {"differing_chunks": diff, "allowed_chunks": allowed, "chunks": entries}
    path = OUT.replace(".json", "_rover.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
