"""Chunk planning on the host, restating the reference pipeline's
planner so that the batched GPU decode receives the same independent units.

  merge_vad_gaps        core/asr_engine.py:2115-2128  (VAD segments closer than 5 s merge)
  concat_speech         core/asr_engine.py:617-644    (speech-only signal + offset map)
  concat_to_original    core/asr_engine.py:647-677    (timestamp map back)
  silent_regions        core/asr_engine.py:521-554    (10 ms RMS frames < 0.01 for >= 0.3 s)
  best_split            core/asr_engine.py:557-573    (silence midpoint nearest the target)
  plan_from_regions     core/asr_engine.py:2141-2161  (the boundary loop given silent regions)
  plan_chunks           core/asr_engine.py:2137-2161  (~30 s boundaries, 3 s overlap)
  split_long_segment    core/asr_engine.py:582-614    (even split of one long segment)

All positions are sample indices at 16 kHz; returned plans are [(start, end, overlap)].
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

SR = 16000
OVERLAP_SEC = 3.0                    # core/asr_engine.py:33
SEGMENT_SEC = 30                     # :2140
MIN_ADVANCE_SEC = 20                 # :2146 (a split closer than this falls back to the target)
MAX_VAD_GAP_SEC = 5                  # :2117

Span = Tuple[int, int]
Chunk = Tuple[int, int, int]


def merge_vad_gaps(segments: Sequence[Span], max_gap: int = MAX_VAD_GAP_SEC * SR) -> List[Span]:
    """Neighbouring speech segments separated by at most `max_gap` samples become one."""
    out: List[Span] = []
    for s, e in segments:
        if out and s - out[-1][1] <= max_gap:
            out[-1] = (out[-1][0], e)
        else:
            out.append((s, e))
    return out


def concat_speech(audio: np.ndarray, segments: Sequence[Span]):
    """Speech-only concatenation and its offset map [(concat_start, orig_start, length)]."""
    if not segments:
        return audio.copy(), [(0, 0, len(audio))]
    parts, omap, pos = [], [], 0
    for s, e in segments:
        omap.append((pos, s, e - s))
        parts.append(audio[s:e])
        pos += e - s
    return np.concatenate(parts), omap


def concat_to_original(t_sec: float, omap, sr: int = SR) -> float:
    """Concat-space seconds -> original seconds (nearest segment edge outside the map)."""
    x = int(t_sec * sr)
    for c0, o0, n in omap:
        if c0 <= x < c0 + n:
            return (o0 + x - c0) / sr
    if omap:
        if x < omap[0][0]:
            return omap[0][1] / sr
        return (omap[-1][1] + omap[-1][2]) / sr
    return t_sec


def silent_regions(audio: np.ndarray, sr: int = SR, threshold: float = 0.01,
                   min_silence: float = 0.3) -> List[Span]:
    """Runs of 10 ms frames with RMS < threshold lasting >= min_silence, in samples."""
    flen = int(sr * 0.01)
    nf = len(audio) // flen
    if nf == 0:
        return []
    rms = np.sqrt(np.mean(audio[:nf * flen].reshape(nf, flen) ** 2, axis=1))
    return regions_from_flags(rms < threshold, flen, len(audio), min_silence)


def regions_from_flags(quiet: np.ndarray, flen: int, n: int, min_silence: float = 0.3) -> List[Span]:
    """The region tail of find_silent_regions (core/asr_engine.py:536-554) given the per-frame
    flags `energies < threshold` (host numpy, or zasr_silence_flags on the device)."""
    if len(quiet) == 0:
        return []
    q = np.concatenate([[False], np.asarray(quiet, bool), [False]]).astype(np.int8)
    edges = np.diff(q)
    starts = np.flatnonzero(edges == 1)          # first quiet frame
    ends = np.flatnonzero(edges == -1)           # one past the last quiet frame
    need = int(min_silence / 0.01)
    keep = (ends - starts) >= need
    return list(zip((starts[keep] * flen).tolist(), np.minimum(ends[keep] * flen, n).tolist()))


def best_split(target: int, total: int, regions: Sequence[Span], window: int = 2 * SR) -> int:
    """Midpoint of the silent region nearest `target` among those touching the +-window;
    `target` itself when none does (ties keep the earlier region)."""
    lo, hi = max(0, target - window), min(total, target + window)
    best, dist = target, math.inf
    for s, e in regions:
        if e >= lo and s <= hi:
            mid = (s + e) // 2
            if abs(mid - target) < dist:
                best, dist = mid, abs(mid - target)
    return best


def plan_from_regions(total: int, regions: Sequence[Span], best_split_fn=None,
                      overlap_sec: float = OVERLAP_SEC, sr: int = SR) -> List[Chunk]:
    """The reference's chunk loop over a signal of `total` samples given its silent regions
    (core/asr_engine.py:2141-2161; `best_split_fn(target, total, regions)` is its
    find_best_split_point, this module's best_split by default): [(start, end, overlap)]."""
    split_at = best_split if best_split_fn is None else best_split_fn
    seg = SEGMENT_SEC * sr
    bounds = [0]
    cur = 0
    while cur + seg < total:
        split = split_at(cur + seg, total, regions)
        if split <= cur + MIN_ADVANCE_SEC * sr:
            split = cur + seg
        bounds.append(split)
        cur = split
    bounds.append(total)
    ov = int(overlap_sec * sr)
    plan: List[Chunk] = []
    for i, (a, b) in enumerate(zip(bounds[:-1], bounds[1:])):
        s = a if i == 0 else max(0, a - ov)
        plan.append((s, b, a - s))
    return plan


def plan_chunks(audio: np.ndarray, sr: int = SR, overlap_sec: float = OVERLAP_SEC) -> List[Chunk]:
    """Silence-aligned ~30 s boundaries over (concatenated) speech; every chunk after the first
    starts `overlap_sec` before its logical start: [(start, end, overlap_at_start)]."""
    return plan_from_regions(len(audio), silent_regions(audio, sr), None, overlap_sec, sr)


def split_long_segment(start: int, end: int, max_sec: float = 30, overlap_sec: float = 3.0,
                       sr: int = SR) -> List[Chunk]:
    """One segment longer than max_sec -> n = ceil(dur / max_sec) equal chunks overlapping by
    overlap_sec (the last one reaches the segment end)."""
    dur = (end - start) / sr
    if dur <= max_sec:
        return [(start, end, 0)]
    n = math.ceil(dur / max_sec)
    clen = int(((dur + (n - 1) * overlap_sec) / n) * sr)
    step = clen - int(overlap_sec * sr)
    out: List[Chunk] = []
    for i in range(n):
        s = start + i * step
        e = end if i == n - 1 else min(s + clen, end)
        out.append((s, e, 0 if i == 0 else int(overlap_sec * sr)))
    return out
