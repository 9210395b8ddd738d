"""ORACLE (test infrastructure only) — CAM++ speaker embedding and its fbank, restated.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

  campp_fbank(audio)      core/speaker_diarization_senko_campp_optimized.py:86-159
                          (_compute_fbank_vectorized: x 32768, snip_edges framing, per-frame DC
                          removal, pre-emphasis whose first sample uses the previous SIGNAL
                          sample (0 for frame 0), Povey window, |rfft 512|^2, 80 kaldi mel bins
                          20 Hz .. Nyquist, floor 1.0, log, per-utterance mean subtraction)
  kaldi_mel_bank()        the 80 x 257 matrix that code takes from kaldi_native_fbank
                          (MelBanks, low 20, high 0 -> Nyquist): triangles linear in mel
                          1127 ln(1 + f / 700), FFT bins 0..255 (column 256 zero).  3P,
                          kaldi-native-fbank is absent: parity of this matrix is unpinned
  CamppOracle.embed(x)    convert_onnx/export_campplus_onnx.py:17-270 (CAMPPlus, eval mode):
                          FCM head (conv / BN / ReLU, BasicResBlocks with (2, 1) strides),
                          TDNN (k 5, stride 2), three CAM dense TDNN blocks with transit
                          layers, BN-ReLU, statistics pooling (mean, unbiased std), dense +
                          affine-free BN.  x: (N, T, 80) -> (N, 192)

Pinned: tests/golden/make_golden_campp.py runs the reference's own CAMPPlus class and its
_compute_fbank_vectorized (with this mel matrix injected: kaldi_native_fbank is absent) on
seeded inputs; tests/test_campp_oracle.py checks this restatement against those outputs.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

BN_EPS = 1e-5


def kaldi_mel_bank(num_bins: int = 80, low: float = 20.0, high: float = 0.0, sr: int = 16000,
                   n_fft: int = 512) -> np.ndarray:
    nyq = 0.5 * sr
    if high <= 0.0:
        high = nyq + high
    mel = lambda f: 1127.0 * math.log(1.0 + f / 700.0)  # noqa: E731
    ml, mh = mel(low), mel(high)
    delta = (mh - ml) / (num_bins + 1)
    width = sr / n_fft
    out = np.zeros((num_bins, n_fft // 2 + 1), dtype=np.float32)
    for b in range(num_bins):
        left, center, right = ml + b * delta, ml + (b + 1) * delta, ml + (b + 2) * delta
        for i in range(n_fft // 2):
            m = mel(width * i)
            if left < m < right:
                out[b, i] = (m - left) / (center - left) if m <= center else (right - m) / (right - center)
    return out


_MEL = None
_WIN = None


def campp_fbank(audio: np.ndarray) -> np.ndarray:
    """(n_frames, 80) float32 with per-utterance CMVN; n_frames = 1 + (N - 400) // 160."""
    global _MEL, _WIN
    if _MEL is None:
        _MEL = kaldi_mel_bank()
        hann = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(400) / 399)
        _WIN = np.power(hann, 0.85).astype(np.float32)
    x = np.asarray(audio, np.float32) * np.float32(32768.0)
    n = x.shape[0]
    if n < 400:
        return np.empty((0, 80), np.float32)
    nf = 1 + (n - 400) // 160
    idx = 160 * np.arange(nf)[:, None] + np.arange(400)[None, :]
    fr = x[idx].astype(np.float32)
    fr -= fr.mean(axis=1, keepdims=True)
    starts = 160 * np.arange(nf)
    ctx = np.where(starts > 0, x[np.maximum(starts - 1, 0)], np.float32(0.0)).astype(np.float32)
    fr[:, 1:] -= np.float32(0.97) * fr[:, :-1]
    fr[:, 0] -= np.float32(0.97) * ctx
    fr *= _WIN
    pad = np.zeros((nf, 512), np.float32)
    pad[:, :400] = fr
    spec = np.fft.rfft(pad)
    power = np.real(spec) ** 2 + np.imag(spec) ** 2
    mel = np.maximum(power @ _MEL.T, 1.0)
    out = np.log(mel).astype(np.float32)
    out -= out.mean(axis=0, keepdims=True)
    return out


class CamppOracle:
    """Eval-mode CAMPPlus forward from a state dict (zasr/campp.py names), torch fp32 (the
    reference's precision) or, with dtype=np.float64, in double as an exact yardstick."""

    def __init__(self, cfg, weights: Dict[str, np.ndarray], dtype=np.float32):
        self.cfg = cfg
        self.dtype = dtype
        self.w = {k: torch.from_numpy(np.asarray(v, dtype)) for k, v in weights.items()}

    def _bn(self, x, name, affine=True):
        w = self.w
        shape = (1, -1) + (1,) * (x.dim() - 2)
        y = (x - w[name + ".running_mean"].view(shape)) / torch.sqrt(w[name + ".running_var"].view(shape) + BN_EPS)
        if affine:
            y = y * w[name + ".weight"].view(shape) + w[name + ".bias"].view(shape)
        return y

    def _resblock(self, x, p, stride):
        w = self.w
        out = F.relu(self._bn(F.conv2d(x, w[p + "conv1.weight"], stride=(stride, 1), padding=1), p + "bn1"))
        out = self._bn(F.conv2d(out, w[p + "conv2.weight"], padding=1), p + "bn2")
        sc = x
        if p + "shortcut.0.weight" in w:
            sc = self._bn(F.conv2d(x, w[p + "shortcut.0.weight"], stride=(stride, 1)), p + "shortcut.1")
        return F.relu(out + sc)

    def _cam(self, x, p, dil):
        w, cfg = self.w, self.cfg
        k = w[p + "linear_local.weight"].shape[-1]
        y = F.conv1d(x, w[p + "linear_local.weight"], padding=(k - 1) // 2 * dil, dilation=dil)
        L = cfg.seg_len
        seg = F.avg_pool1d(x, kernel_size=L, stride=L, ceil_mode=True)
        seg = seg.unsqueeze(-1).expand(*seg.shape, L).reshape(*seg.shape[:-1], -1)[..., :x.shape[-1]]
        ctx = x.mean(-1, keepdim=True) + seg
        ctx = F.relu(F.conv1d(ctx, w[p + "linear1.weight"], w[p + "linear1.bias"]))
        m = torch.sigmoid(F.conv1d(ctx, w[p + "linear2.weight"], w[p + "linear2.bias"]))
        return y * m

    def embed(self, feats: np.ndarray) -> np.ndarray:
        cfg, w = self.cfg, self.w
        with torch.no_grad():
            x = torch.from_numpy(np.asarray(feats, self.dtype)).permute(0, 2, 1).unsqueeze(1)
            x = F.relu(self._bn(F.conv2d(x, w["head.conv1.weight"], padding=1), "head.bn1"))
            for li, nb in enumerate(cfg.head_blocks):
                for b in range(nb):
                    x = self._resblock(x, f"head.layer{li + 1}.{b}.", 2 if b == 0 else 1)
            x = F.relu(self._bn(F.conv2d(x, w["head.conv2.weight"], stride=(2, 1), padding=1), "head.bn2"))
            x = x.reshape(x.shape[0], x.shape[1] * x.shape[2], x.shape[3])
            x = F.conv1d(x, w["xvector.tdnn.linear.weight"], stride=2, padding=2)
            x = F.relu(self._bn(x, "xvector.tdnn.nonlinear.batchnorm"))
            for bi, (nl, dil) in enumerate(zip(cfg.block_layers, cfg.block_dilations)):
                for i in range(nl):
                    p = f"xvector.block{bi + 1}.tdnnd{i + 1}."
                    h = F.conv1d(F.relu(self._bn(x, p + "nonlinear1.batchnorm")), w[p + "linear1.weight"])
                    h = F.relu(self._bn(h, p + "nonlinear2.batchnorm"))
                    x = torch.cat([x, self._cam(h, p + "cam_layer.", dil)], dim=1)
                p = f"xvector.transit{bi + 1}."
                x = F.conv1d(F.relu(self._bn(x, p + "nonlinear.batchnorm")), w[p + "linear.weight"])
            x = F.relu(self._bn(x, "xvector.out_nonlinear.batchnorm"))
            x = torch.cat([x.mean(-1), x.std(-1, unbiased=True)], dim=-1)
            x = F.conv1d(x.unsqueeze(-1), w["xvector.dense.linear.weight"]).squeeze(-1)
            x = self._bn(x, "xvector.dense.nonlinear.batchnorm", affine=False)
        return x.numpy().astype(np.float32)
