"""Chunk-overlap merge of the decoded word lists (host side, after the GPU decode).

The reference plans ~30 s chunks with 3 s of overlap (zasr.plan) and, once every chunk is
decoded, stitches their word lists: the words of chunk k-1 that start inside its last
`overlap` seconds (tail) are aligned against the words of chunk k that start inside its first
`overlap` seconds (head) by a sliding offset with fuzzy word equality; a good alignment cuts
the head's duplicate words (and pops tail words past the last match), no alignment drops the
less confident side.  Restated from core/asr_engine.py:44-237 (normalize_word_for_overlap,
words_match, find_overlap_alignment, merge_chunks_with_overlap); pinned by
tests/golden/merge_cases.json, made by running those reference functions
(tests/golden/make_golden_merge.py).
"""
from __future__ import annotations

import re
import unicodedata
from difflib import SequenceMatcher
from functools import lru_cache
from typing import Dict, List, Sequence, Tuple

OVERLAP_SEC = 3.0           # core/asr_engine.py:33
MAX_OVERLAP_WORDS = 100     # :35
FUZZY_MATCH_THRESHOLD = 0.8  # :36
MIN_MATCH_RATIO = 0.5       # :37

_NON_WORD = re.compile(r"[^\w]", flags=re.UNICODE)


def overlap_key(text: str) -> str:
    """Comparison form of a word (:44-49): lower-case, NFC, word characters only."""
    return _NON_WORD.sub("", unicodedata.normalize("NFC", text.lower().strip()))


@lru_cache(maxsize=1 << 16)
def fuzzy_equal(a: str, b: str, threshold: float = FUZZY_MATCH_THRESHOLD) -> bool:
    """:52-67: identical, one containing the other (both longer than 2), or a difflib ratio
    of at least `threshold` (quick_ratio bounds ratio from above: below the threshold it
    decides without the matching-block search)."""
    if a == b:
        return True
    if not a or not b:
        return False
    if len(a) > 2 and len(b) > 2 and (a in b or b in a):
        return True
    sm = SequenceMatcher(None, a, b)
    return sm.quick_ratio() >= threshold and sm.ratio() >= threshold


def _mean_prob(ws: Sequence[Dict]) -> float:
    return sum(w.get("prob", 1.0) for w in ws) / max(1, len(ws))


def align_overlap(tail: Sequence[Dict], head: Sequence[Dict]) -> Tuple[int, str, int]:
    """(first head index to keep, action, tail words to pop) -- :70-179.

    Every offset of the (at most 100-word) tail against the head is scored by its count of
    fuzzy-equal pairs; the best offset with a match ratio >= 0.5 over its overlap window wins
    (first best on ties).  Without a match, or when the best alignment is shorter than the
    shorter side and leaves unmatched tail words, the divergent parts' mean probabilities
    decide which side is dropped."""
    if not tail or not head:
        return 0, "none", 0
    tk = [overlap_key(w["text"]) for w in tail[-MAX_OVERLAP_WORDS:]]
    hk = [overlap_key(w["text"]) for w in head[:MAX_OVERLAP_WORDS]]
    nt, nh = len(tk), len(hk)
    best, cut, pop = 0, 0, 0
    for off in range(1 - nt, nh):
        lo, hi = max(0, -off), min(nt, nh - off)  # tail indices i with 0 <= i + off < nh
        hits = [i for i in range(lo, hi) if fuzzy_equal(tk[i], hk[i + off])]
        window = min(nh, nt + off) - max(0, off)
        if len(hits) > best and len(hits) / max(1, window) >= MIN_MATCH_RATIO:
            best = len(hits)
            cut = hits[-1] + off + 1
            pop = nt - 1 - hits[-1]
    if best == 0 or (best < min(nt, nh) and pop > 0):
        if best == 0:
            d_tail, d_head = list(tail), list(head)
        else:
            d_tail = list(tail[-pop:]) if pop > 0 else []
            d_head = list(head[cut:]) if cut < len(head) else []
        if _mean_prob(d_tail) > _mean_prob(d_head):
            return len(head), "drop_head", 0
        return 0, "drop_tail", len(tail)
    return cut, "cut_head", pop


def merge_chunks_with_overlap(chunk_results: Sequence[Dict], overlap_sec: float = OVERLAP_SEC
                              ) -> Tuple[List[Dict], str]:
    """:182-237.  chunk_results: dicts with "words" (each with local_start), "audio_start_abs"
    and "audio_end_abs"; returns (merged word dicts, their texts joined by spaces)."""
    merged: List[Dict] = []
    for k, chunk in enumerate(chunk_results):
        words = chunk["words"]
        if k == 0:
            merged.extend(words)
            continue
        prev = chunk_results[k - 1]
        tail_from = max(0, (prev["audio_end_abs"] - prev["audio_start_abs"]) - overlap_sec)
        tail = [w for w in prev["words"] if w.get("local_start", 0) >= tail_from]
        head = [w for w in words if w.get("local_start", 0) < overlap_sec]
        cut, _, pop = align_overlap(tail, head)
        if pop > 0:
            del merged[-pop:]
        merged.extend(words[cut:] if cut < len(words) else [])
    return merged, " ".join(w["text"] for w in merged)
