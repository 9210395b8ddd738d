"""Golden fixtures for the host-side planner and the ROVER block vote
(row L), produced by running the REFERENCE's own functions.

Run in the build container only (needs /root/reference; the GPU box never runs this):

    python tests/golden/make_golden_host.py

Reference functions driven: core/asr_engine.py find_silent_regions (:521),
find_best_split_point (:557), chunk_long_segment (:582), map_concat_time_to_original (:647),
rover_merge_words (:1446, with its hotword phrase cache set from tests/golden/hotword_sample.txt,
the reference's hotword.txt data).  The ~30 s planner loop itself is inline in
TranscriberPipeline.run (:2137-2157); it is re-driven here around the reference helpers.

Outputs: tests/golden/plan_cases.json, tests/golden/rover_cases.json.
"""
from __future__ import annotations

import contextlib
import copy
import hashlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "sherpa-vietnamese-asr_amd"))
REF = "/root/reference"
HOTWORDS = os.path.join(HERE, "hotword_sample.txt")


def _ref():
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import core.asr_engine as ae
        import core.hotword_context as hc
    return ae, hc


def plan_audio(seed: int, seconds: float) -> np.ndarray:
    from zasr.synth_audio import synth_speech
    return synth_speech(seconds, seed)


def audio_sum(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()[:16]


def make_plans(ae):
    cases = []
    for seed, sec in ((11, 95.0), (12, 181.5), (13, 62.0), (14, 29.0)):
        a = plan_audio(seed, sec)
        regions = ae.find_silent_regions(a)
        total = len(a)
        seg = 16000 * 30
        bounds, cur = [0], 0
        while cur + seg < total:
            best = ae.find_best_split_point(cur + seg, total, regions)
            if best <= cur + 20 * 16000:
                best = cur + seg
            bounds.append(best)
            cur = best
        bounds.append(total)
        plan = []
        for i in range(len(bounds) - 1):
            s = bounds[i] if i == 0 else max(0, bounds[i] - ae.OVERLAP_SAMPLES)
            plan.append([s, bounds[i + 1], bounds[i] - s])
        cases.append({"seed": seed, "seconds": sec, "audio_sha": audio_sum(a),
                      "silent_regions": [list(map(int, r)) for r in regions],
                      "plan": [list(map(int, p)) for p in plan]})
    long_segs = []
    for s, e in ((0, 16000 * 29), (5000, 5000 + 16000 * 31), (100, 100 + 16000 * 95 + 7),
                 (0, 16000 * 61)):
        long_segs.append({"start": s, "end": e,
                          "chunks": [list(map(int, c)) for c in ae.chunk_long_segment(s, e)]})
    omap = [(0, 16000 * 2, 16000 * 5), (16000 * 5, 16000 * 9, 16000 * 3),
            (16000 * 8, 16000 * 20, 16000 * 4)]
    times = [0.0, 1.25, 4.999, 5.0, 7.5, 8.0, 11.9, 12.0, 15.0, -0.5]
    mapped = [ae.map_concat_time_to_original(t, omap) for t in times]
    return {"cases": cases, "long_segments": long_segs,
            "concat_map": {"offset_map": omap, "times": times, "original": mapped}}


SYLS = ["xin", "chào", "các", "bạn", "hôm", "nay", "chúng", "ta", "sẽ", "nói", "về", "công",
        "nghệ", "trí", "tuệ", "nhân", "tạo", "và", "ứng", "dụng", "trong", "đời", "sống", "ban",
        "tổ", "chức", "hội", "nghị", "việt", "nam", "hà", "nội", "thành", "phố", "hồ", "chí",
        "minh", "kinh", "tế", "xã", "đang", "phát", "triển", "mạnh", "mẽ"]


def rand_word(rng, t, text=None):
    return {"text": text if text is not None else SYLS[int(rng.integers(len(SYLS)))],
            "start": round(float(t), 3), "end": round(float(t) + 0.2, 3),
            "prob": round(float(rng.uniform(0.3, 1.0)), 4),
            "tsallis_max": round(float(rng.uniform(0.0, 0.9)), 4),
            "margin_min": round(float(rng.uniform(0.0, 1.0)), 4),
            "entropy_norm": round(float(rng.uniform(0.0, 0.8)), 4)}


def make_rover(ae, hc):
    phrases = [p for p, _ in hc.parse_hotwords_file(HOTWORDS)]
    ae._hotword_phrases_cache = sorted([p.lower() for p in phrases], key=len, reverse=True)
    rng = np.random.Generator(np.random.PCG64(20261015))
    cases = []
    for k in range(40):
        n = int(rng.integers(0, 40))
        t = 0.0
        A = []
        for _ in range(n):
            t += float(rng.uniform(0.1, 0.5))
            A.append(rand_word(rng, t))
        if k % 5 == 1 and n > 4:  # plant a hotword phrase in A or B
            ph = phrases[int(rng.integers(len(phrases)))].split()
            pos = int(rng.integers(0, n - 1))
            for q, syl in enumerate(ph):
                if pos + q < n:
                    A[pos + q]["text"] = syl.lower()
        B = []
        for w in A:
            u = float(rng.uniform())
            if u < 0.12:
                continue                                   # deletion
            nw = dict(w)
            for key in ("prob", "tsallis_max", "margin_min"):
                nw[key] = round(float(np.clip(w[key] + rng.normal(0, 0.2), 0.0, 1.0)), 4)
            if u < 0.30:
                nw["text"] = SYLS[int(rng.integers(len(SYLS)))]  # substitution
            B.append(nw)
            if float(rng.uniform()) < 0.10:                 # insertion (maybe a near-duplicate)
                ins = rand_word(rng, w["start"] + float(rng.choice([0.05, 0.1, 0.3])),
                                text=w["text"] if float(rng.uniform()) < 0.5 else None)
                B.append(ins)
        if k % 7 == 3:
            for w in B:
                w.pop("margin_min")
        if k == 5:
            A = []
        if k == 6:
            B = []
        with contextlib.redirect_stdout(io.StringIO()):
            merged, dis = ae.rover_merge_words(copy.deepcopy(A), copy.deepcopy(B))
        cases.append({"A": A, "B": B, "merged": merged, "disagree": sorted(dis)})
    return {"hotword_phrases": phrases, "cases": cases}


def main():
    ae, hc = _ref()
    with open(os.path.join(HERE, "plan_cases.json"), "w") as f:
        json.dump(make_plans(ae), f, ensure_ascii=False)
    with open(os.path.join(HERE, "rover_cases.json"), "w") as f:
        json.dump(make_rover(ae, hc), f, ensure_ascii=False)
    print("wrote plan_cases.json, rover_cases.json")


if __name__ == "__main__":
    main()
