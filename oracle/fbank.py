"""ORACLE (test infrastructure only) — numpy restatement of the reference's fbank.

Reference call site: `core/asr_engine.py:698-721` (`compute_fbank_ort`), which runs
kaldi-native-fbank `OnlineFbank` (3P, unpinned version, not installed offline) with
dither=0, snip_edges=False, 16 kHz, 25 ms / 10 ms, povey window, 80 mel bins 20..7600 Hz,
energy_floor=1 (unused: use_energy=False), samples in [-1, 1] (no x32768).

Restated kaldi semantics:
  frames      T = (N + 80) // 160; frame f starts at 160 f - 120, indices reflected
  per frame   remove DC (f32), pre-emphasis 0.97 (i = 399..1, then w0 -= 0.97 w0),
              povey window (0.5 - 0.5 cos(2 pi i / 399))^0.85, zero-pad to 512,
              real FFT (knf computes its rdft in double), power |X_k|^2 (f32),
              mel: 80 triangles linear in mel = 1127 ln(1 + f/700) over FFT bins 0..255,
              log(max(e, FLT_EPSILON)).

PARITY: kaldi-native-fbank itself is absent, but the reference ships a second, executable
fbank -- `computeFbank`, `offline_pwa/static/js/pure-ort-asr-worker.js:470-519` -- and
tests/golden/make_golden_fbank_js.py runs it under node.  `fbank_js` below restates that
function (f64 framing / FFT / power / mel sums, f32 window and triangle weights, triangles
linear in Hz incl. the Nyquist bin, log floor 2^-23) and is pinned to its outputs within 1e-5
(tests/test_fbank_oracle.py).  `fbank` (the GPU's target, knf's semantics) shares every step
with it except the two documented ones: triangles linear in mel over bins 0..255 (knf's
MelBanks) and the f32 DC removal / pre-emphasis / window / power of knf's float pipeline; the
tests bound that difference on the same fixtures.  The mel-vs-Hz triangle choice is the one
step no reference-run output pins.
"""
from __future__ import annotations

import numpy as np

FRAME_LEN = 400
FRAME_SHIFT = 160
NFFT = 512
NUM_BINS = 80
LOW_FREQ = 20.0
HIGH_FREQ = 7600.0
PREEMPH = np.float32(0.97)
FLT_EPS = np.float32(np.finfo(np.float32).eps)


def num_frames(n: int) -> int:
    return (n + FRAME_SHIFT // 2) // FRAME_SHIFT if n > 0 else 0


def povey_window() -> np.ndarray:
    i = np.arange(FRAME_LEN, dtype=np.float64)
    a = 2.0 * np.pi / (FRAME_LEN - 1)
    return np.power(0.5 - 0.5 * np.cos(a * i), 0.85).astype(np.float32)


def _mel(f):
    f = np.asarray(f, dtype=np.float32)
    return np.float32(1127.0) * np.log(np.float32(1.0) + f / np.float32(700.0))  # kaldi MelScale (logf)


def mel_banks() -> np.ndarray:
    """(80, 256) float32 weights, kaldi MelBanks with mel-domain triangles."""
    nbins = NFFT // 2
    bin_w = np.float32(16000.0 / NFFT)
    mel_lo, mel_hi = _mel(LOW_FREQ), _mel(HIGH_FREQ)
    delta = (mel_hi - mel_lo) / np.float32(NUM_BINS + 1)
    mels = _mel(bin_w * np.arange(nbins, dtype=np.float32))
    W = np.zeros((NUM_BINS, nbins), dtype=np.float32)
    for b in range(NUM_BINS):
        left = mel_lo + np.float32(b) * delta
        center = mel_lo + np.float32(b + 1) * delta
        right = mel_lo + np.float32(b + 2) * delta
        up = (mels > left) & (mels <= center)
        dn = (mels > center) & (mels < right)
        W[b, up] = (mels[up] - left) / (center - left)
        W[b, dn] = (right - mels[dn]) / (right - center)
    return W


def frame_indices(n: int) -> np.ndarray:
    """(T, 400) int64 sample indices with kaldi's repeated edge reflection."""
    T = num_frames(n)
    idx = (np.arange(T, dtype=np.int64)[:, None] * FRAME_SHIFT
           - (FRAME_LEN - FRAME_SHIFT) // 2 + np.arange(FRAME_LEN, dtype=np.int64)[None, :])
    for _ in range(64):
        neg = idx < 0
        big = idx >= n
        if not (neg.any() or big.any()):
            break
        idx = np.where(neg, -idx - 1, idx)
        idx = np.where(big, 2 * n - 1 - idx, idx)
    return idx


def fbank(audio: np.ndarray, banks: np.ndarray = None) -> np.ndarray:
    """audio float32 [N] in [-1, 1] -> float32 [T, 80] log-mel (kaldi semantics).  `banks`
    (checker use): other (80, 257) triangles in place of mel_banks(), e.g. mel_banks_js() to
    isolate the triangle difference against the reference's executable fbank."""
    audio = np.asarray(audio, dtype=np.float32)
    n = audio.shape[0]
    T = num_frames(n)
    if T == 0:
        return np.zeros((0, NUM_BINS), dtype=np.float32)
    frames = audio[frame_indices(n)].astype(np.float32)  # (T, 400)
    mean = (frames.astype(np.float64).sum(axis=1) / FRAME_LEN).astype(np.float32)
    frames = frames - mean[:, None]
    prev = np.concatenate([frames[:, :1], frames[:, :-1]], axis=1)
    frames = frames - PREEMPH * prev
    frames = frames * povey_window()[None, :]
    spec = np.fft.rfft(frames.astype(np.float64), n=NFFT, axis=1)  # double, like knf rdft
    re = spec.real.astype(np.float32)
    im = spec.imag.astype(np.float32)
    power = re * re + im * im  # (T, 257) float32
    if banks is None:
        mel = power[:, : NFFT // 2] @ mel_banks().T.astype(np.float32)
    else:
        mel = power @ banks.T.astype(np.float32)
    return np.log(np.maximum(mel, FLT_EPS)).astype(np.float32)


def _hz_of_mel(m):
    return 700.0 * (np.exp(m / 1127.0) - 1.0)


def mel_banks_js() -> np.ndarray:
    """(80, 257) float32: pure-ort-asr-worker.js:369-397 -- centres evenly spaced in mel,
    triangles linear in Hz over bins 0..256 (f64 arithmetic, Float32Array storage)."""
    mel = lambda f: 1127.0 * np.log(1.0 + f / 700.0)
    lo, hi = mel(LOW_FREQ), mel(HIGH_FREQ)
    delta = (hi - lo) / (NUM_BINS + 1)
    centers = _hz_of_mel(lo + np.arange(NUM_BINS + 2, dtype=np.float64) * delta)
    freqs = np.arange(NFFT // 2 + 1, dtype=np.float64) * 16000.0 / NFFT
    W = np.zeros((NUM_BINS, NFFT // 2 + 1), dtype=np.float64)
    for m in range(NUM_BINS):
        left, center, right = centers[m], centers[m + 1], centers[m + 2]
        up = (freqs > left) & (freqs <= center)
        dn = (freqs > center) & (freqs < right)
        W[m, up] = (freqs[up] - left) / max(center - left, 1e-12)
        W[m, dn] = (right - freqs[dn]) / max(right - center, 1e-12)
    return W.astype(np.float32)


def fbank_js(audio: np.ndarray) -> np.ndarray:
    """The reference's executable fbank (pure-ort-asr-worker.js:470-519) restated: frames of
    reflected samples (:460-468, :485-491), f64 DC removal and pre-emphasis times the f32
    window (:494-500), f64 FFT power (:502-505), f64 sums over the f32 Hz triangles and
    log(max(e, 2^-23)) stored as f32 (:507-515)."""
    audio = np.asarray(audio, dtype=np.float32)
    n = audio.shape[0]
    T = num_frames(n)
    if T == 0:
        return np.zeros((0, NUM_BINS), dtype=np.float32)
    fr = audio[frame_indices(n)].astype(np.float64)
    fr = fr - fr.sum(axis=1, keepdims=True) / FRAME_LEN
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    x = (fr - 0.97 * prev) * povey_window().astype(np.float64)[None, :]
    spec = np.fft.rfft(x, n=NFFT, axis=1)
    power = spec.real * spec.real + spec.imag * spec.imag
    e = power @ mel_banks_js().astype(np.float64).T
    return np.log(np.maximum(e, 1.1920928955078125e-7)).astype(np.float32)
