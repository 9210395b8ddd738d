"""Seeded synthetic 16 kHz "speech" (SURVEY §8d "Synthetic input").

Glottal pulse train (F0 90-220 Hz) through three formant resonators, 4-6 Hz syllable
envelope, unvoiced noise bursts, 0.3-2 s pauses, peak 0.6-0.9 (so load_audio's low-volume
boost, core/asr_engine.py:512-516, is a no-op).  Chunks follow the reference planner's
shape: ~30 s pieces (20-33 s) with a 3 s overlap (core/asr_engine.py:2137-2161).
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np

SR = 16000


def _resonate(x: np.ndarray, f: float, bw: float) -> np.ndarray:
    r = np.exp(-np.pi * bw / SR)
    a1 = -2 * r * np.cos(2 * np.pi * f / SR)
    a2 = r * r
    y = np.zeros_like(x)
    y1 = y2 = 0.0
    # second-order IIR, vectorised in blocks is not needed at these sizes
    for i in range(x.shape[0]):
        v = x[i] - a1 * y1 - a2 * y2
        y[i] = v
        y2, y1 = y1, v
    return y


def synth_speech(seconds: float, seed: int = 20261015) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    n = int(seconds * SR)
    out = np.zeros(n, dtype=np.float64)
    pos = 0
    while pos < n:
        seg = int(rng.uniform(1.0, 4.0) * SR)
        seg = min(seg, n - pos)
        t = np.arange(seg) / SR
        f0 = rng.uniform(90, 220) * (1 + 0.1 * np.sin(2 * np.pi * rng.uniform(0.5, 2) * t))
        phase = np.cumsum(f0 / SR)
        pulses = (np.diff(np.floor(phase), prepend=0.0) > 0).astype(np.float64)
        src = np.convolve(pulses, np.hanning(24))[:seg]
        src += 0.05 * rng.standard_normal(seg)
        v = np.zeros(seg)
        for fmt, bw in ((rng.uniform(300, 800), 80), (rng.uniform(900, 2200), 120),
                        (rng.uniform(2300, 3200), 180)):
            v += _resonate_fast(src, fmt, bw)
        env = 0.5 * (1 - np.cos(2 * np.pi * rng.uniform(4, 6) * t)) ** 1.5
        burst = (rng.random(seg) < 0.002).astype(np.float64)
        # 400-sample box sum of the burst train (== np.convolve(burst, ones(400))[:seg],
        # exactly: small integers in float64) in O(seg)
        csum = np.cumsum(burst)
        box = csum.copy()
        box[400:] -= csum[:-400]
        noise = box * rng.standard_normal(seg) * 0.3
        out[pos: pos + seg] = v * env + noise
        pos += seg
        pause = int(rng.uniform(0.3, 2.0) * SR)
        pos += pause  # silence (zeros) + very low noise below
    out += 1e-4 * rng.standard_normal(n)
    peak = np.max(np.abs(out))
    out = out / max(peak, 1e-9) * rng.uniform(0.6, 0.9)
    return out.astype(np.float32)


def _resonate_fast(x: np.ndarray, f: float, bw: float) -> np.ndarray:
    """Same resonator as _resonate via scipy's lfilter when available."""
    try:
        from scipy.signal import lfilter
    except Exception:  # pragma: no cover
        return _resonate(x, f, bw)
    r = np.exp(-np.pi * bw / SR)
    return lfilter([1.0], [1.0, -2 * r * np.cos(2 * np.pi * f / SR), r * r], x)


def chunk_plan(total: int, seg_sec: float = 30.0, overlap_sec: float = 3.0,
               min_sec: float = 20.0) -> List[Tuple[int, int, int]]:
    """Fixed-target restatement of the reference planner without silence search:
    boundaries every ~seg_sec, each chunk after the first starts overlap_sec early
    (core/asr_engine.py:2137-2161)."""
    seg, ov = int(seg_sec * SR), int(overlap_sec * SR)
    bounds = [0]
    cur = 0
    while cur + seg < total:
        cur += seg
        bounds.append(cur)
    bounds.append(total)
    if len(bounds) > 2 and bounds[-1] - bounds[-2] < int(min_sec * SR) // 4:
        bounds.pop(-2)
    plan = []
    for i in range(len(bounds) - 1):
        s, e = bounds[i], bounds[i + 1]
        a = s if i == 0 else max(0, s - ov)
        plan.append((a, e, s - a))
    return plan


def synth_chunks(total_seconds: float, seed: int = 20261015) -> List[np.ndarray]:
    audio = synth_speech(total_seconds, seed)
    return [audio[a:e] for a, e, _ in chunk_plan(audio.shape[0])]
