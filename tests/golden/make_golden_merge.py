"""Golden fixtures for the chunk-overlap merge (zasr.merge), produced by running the
REFERENCE's own merge_chunks_with_overlap / find_overlap_alignment
(core/asr_engine.py:70-237) on synthetic chunk word lists.

Run in the build container only (needs /root/reference; the GPU box never runs this):

    python tests/golden/make_golden_merge.py

Output: tests/golden/merge_cases.json -- [{"chunks": [...], "picked": [[chunk, word], ...],
"text": "..."}]: the merged list as (chunk index, word index) pairs into "chunks".
"""
from __future__ import annotations

import contextlib
import copy
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

SYLL = ["xin", "chào", "các", "bạn", "hôm", "nay", "trời", "đẹp", "quá", "chúng", "ta", "đi",
        "học", "Việt", "Nam", "thành", "phố", "Hồ", "Chí", "Minh", "một", "hai", "ba", "người",
        "nói", "được", "không", "này", "đó", "với", "cho", "những", "khi", "đã", "sẽ", "là"]


def _variant(rng, w):
    """A decoding variant of word w inside an overlap region."""
    k = rng.integers(6)
    if k == 0:
        return w.upper()
    if k == 1:
        return w + ","
    if k == 2:
        return w[:-1] if len(w) > 2 else w + "a"
    if k == 3:
        return str(rng.choice(SYLL))
    return w


def _chunks(rng, n_chunks, mode):
    """Chunks of a timeline of words (~0.35 s each): chunk k covers [27k, 27k + 30) s."""
    T = 27.0 * (n_chunks - 1) + 30.0
    n = int(T / 0.35)
    truth = [(str(rng.choice(SYLL)), 0.35 * i + 0.05 * rng.random()) for i in range(n)]
    out = []
    for k in range(n_chunks):
        a, e = 27.0 * k, 27.0 * k + 30.0
        words = []
        for text, t in truth:
            if not (a <= t < e - 0.2):
                continue
            loc = t - a
            in_ov = loc < 3.0 or loc >= 27.0
            if in_ov and mode == "noisy":
                if rng.random() < 0.35:
                    text = _variant(rng, text)
                if rng.random() < 0.1:
                    continue
            if in_ov and mode == "diverge" and loc < 3.0:
                text = str(rng.choice(SYLL)) + "x"
            words.append({"text": text, "local_start": round(loc, 3),
                          "prob": round(float(rng.uniform(0.3, 1.0)), 3)})
        if mode == "empty" and k == 1:
            words = []
        out.append({"words": words, "audio_start_abs": a, "audio_end_abs": e})
    return out


def _run(ae, mode, chunks):
    cp = copy.deepcopy(chunks)
    where = {id(wd): [k, i] for k, c in enumerate(cp) for i, wd in enumerate(c["words"])}
    with contextlib.redirect_stdout(io.StringIO()):
        words, text = ae.merge_chunks_with_overlap(cp)
    return {"mode": mode, "chunks": chunks, "picked": [where[id(wd)] for wd in words], "text": text}


def main():
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import core.asr_engine as ae
    rng = np.random.default_rng(20261017)
    cases = []
    for mode in ("clean", "noisy", "diverge", "empty"):
        for rep in range(6 if mode == "noisy" else 2):
            chunks = _chunks(rng, int(rng.integers(2, 5)), mode)
            cases.append(_run(ae, mode, chunks))
    # hand cases: single chunk, all-empty, tail junk after a match (pop), exact duplicates
    w = lambda t, ls, p=0.9: {"text": t, "local_start": ls, "prob": p}  # noqa: E731
    hand = [
        [{"words": [w("a", 0.1)], "audio_start_abs": 0.0, "audio_end_abs": 30.0}],
        [{"words": [], "audio_start_abs": 0.0, "audio_end_abs": 30.0},
         {"words": [], "audio_start_abs": 27.0, "audio_end_abs": 57.0}],
        [{"words": [w("một", 27.1), w("hai", 27.5), w("ba", 28.0), w("rác", 29.5, 0.2)],
          "audio_start_abs": 0.0, "audio_end_abs": 30.0},
         {"words": [w("một", 0.1), w("hai", 0.5), w("ba", 1.0), w("bốn", 2.0), w("năm", 4.0)],
          "audio_start_abs": 27.0, "audio_end_abs": 57.0}],
        [{"words": [w("xin", 27.2), w("chào", 27.8)], "audio_start_abs": 0.0, "audio_end_abs": 30.0},
         {"words": [w("Xin,", 0.2), w("chào.", 0.8), w("bạn", 3.5)],
          "audio_start_abs": 27.0, "audio_end_abs": 57.0}],
    ]
    for chunks in hand:
        cases.append(_run(ae, "hand", chunks))
    path = os.path.join(HERE, "merge_cases.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump(cases, f, ensure_ascii=False)
    print(f"wrote {len(cases)} cases to {path}")


if __name__ == "__main__":
    main()
