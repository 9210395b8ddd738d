"""fbank oracle self-checks (kaldi-native-fbank itself is absent offline: parity unpinned).

Known answers: frame count (N + 80) // 160 (snip_edges=False); silence -> log(FLT_EPSILON);
a pure tone peaks in the mel bin whose centre is nearest; edge frames use kaldi's
reflection; mel triangles are linear in mel between 20 and 7600 Hz.  Cross-check: the
reference's second restatement (offline_pwa/static/js/pure-ort-asr-worker.js:351-519,
Hz-domain triangles) must agree to within its known triangle-shape difference.
"""
import numpy as np
import pytest

from oracle.fbank import (FLT_EPS, fbank, frame_indices, mel_banks, num_frames, povey_window)


@pytest.mark.parametrize("n,T", [(0, 0), (1, 0), (79, 0), (80, 1), (239, 1), (240, 2),
                                 (16000, 100), (480000, 3000), (480080, 3001)])
def test_frame_count(n, T):
    assert num_frames(n) == T


def test_silence_is_log_eps():
    f = fbank(np.zeros(16000, np.float32))
    assert f.shape == (100, 80)
    assert np.all(f == np.float32(np.log(FLT_EPS)))


def test_reflection_indices():
    idx = frame_indices(1000)
    assert idx[0, 0] == 119  # s = -120 -> -s - 1
    assert idx[0, 120] == 0
    last = idx[-1]
    assert last.max() <= 999 and last.min() >= 0
    # tiny input: repeated reflection stays in range
    assert frame_indices(100).min() >= 0 and frame_indices(100).max() <= 99


def _mel_center_hz(b):
    m = lambda f: 1127.0 * np.log(1 + f / 700.0)
    lo, hi = m(20.0), m(7600.0)
    c = lo + (b + 1) * (hi - lo) / 81
    return 700.0 * (np.exp(c / 1127.0) - 1)


@pytest.mark.parametrize("b", [5, 20, 40, 60, 75])
def test_tone_peaks_in_its_bin(b):
    f0 = _mel_center_hz(b)
    t = np.arange(16000) / 16000.0
    f = fbank((0.5 * np.sin(2 * np.pi * f0 * t)).astype(np.float32))
    assert abs(int(np.argmax(f[50])) - b) <= 1


def test_mel_banks_shape_and_partition():
    W = mel_banks()
    assert W.shape == (80, 256)
    assert np.all(W >= 0) and np.all(W <= 1)
    # adjacent triangles sum to ~1 between the first and last centres
    s = W.sum(axis=0)
    inner = s[20:230]
    assert np.all(np.abs(inner[inner > 0] - 1.0) < 1e-4)


def test_povey_window():
    w = povey_window()
    assert w.shape == (400,) and w[0] == 0.0 and abs(w[199] - 1.0) < 1e-4


def _js_style_fbank(audio):
    """numpy transcription of the PWA worker's computeFbank (Hz-domain triangles,
    radix-2 FFT incl. the Nyquist bin) — loose cross-check only."""
    n = audio.shape[0]
    T = num_frames(n)
    idx = frame_indices(n)
    win = povey_window().astype(np.float64)
    hz = lambda m: 700.0 * (np.exp(m / 1127.0) - 1.0)
    mel = lambda f: 1127.0 * np.log(1.0 + f / 700.0)
    lo, hi = mel(20.0), mel(7600.0)
    centers = hz(lo + np.arange(82) * (hi - lo) / 81)
    freqs = np.arange(257) * 16000.0 / 512
    W = np.zeros((80, 257))
    for m in range(80):
        l, c, r = centers[m], centers[m + 1], centers[m + 2]
        up = (freqs > l) & (freqs <= c)
        dn = (freqs > c) & (freqs < r)
        W[m, up] = (freqs[up] - l) / (c - l)
        W[m, dn] = (r - freqs[dn]) / (r - c)
    fr = audio[idx].astype(np.float64)
    fr -= fr.mean(axis=1, keepdims=True)
    prev = np.concatenate([fr[:, :1], fr[:, :-1]], axis=1)
    x = (fr - 0.97 * prev) * win
    p = np.abs(np.fft.rfft(x, 512)) ** 2
    return np.log(np.maximum(p @ W.T, 1.1920929e-07)).astype(np.float32)


def test_cross_check_with_reference_js_restatement():
    rng = np.random.default_rng(1)
    a = (0.3 * rng.standard_normal(16000 * 2)).astype(np.float32)
    ours, js = fbank(a), _js_style_fbank(a)
    # triangles differ (mel- vs Hz-linear); broadband noise keeps the bins close
    assert np.median(np.abs(ours - js)) < 0.05
    assert np.max(np.abs(ours - js)) < 0.5
