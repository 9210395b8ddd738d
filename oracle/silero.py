"""ORACLE (test infrastructure only) — Silero VAD restated in torch fp32, plus the
reference's VAD window loop and segmentation.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

  SileroOracle.window     the silero-vad v5 16 kHz network (third-party, see zasr/silero.py),
                          one call = what the reference's session.run does per window
  SileroOracle.session    an object with the onnxruntime run(None, feeds) surface
  run_windows             core/vad_utils.py:80-111   (64-sample context, carried state)
  speech_windows          core/vad_utils.py:120-151  (threshold / min silence / min speech)
  vad_segments            core/vad_utils.py:158-260  (boost, retry at 0.3, fallback, padding,
                                                      merge)

The loop and segmentation are pinned by tests/golden/make_golden_vad.py, which runs the
reference's own vad_utils functions with this network behind its session.  The network
itself is parity-unpinned against the real silero_vad_16k_op15.onnx (not present).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch
import torch.nn.functional as F

WINDOW, CONTEXT = 512, 64


class SileroOracle:
    def __init__(self, cfg, weights: Dict[str, np.ndarray]):
        self.cfg = cfg
        self.w = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in weights.items()}

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        """[N, 576] -> encoder output [N, 128] (STFT magnitude + 4 conv blocks)."""
        cfg, w = self.cfg, self.w
        xp = F.pad(x[:, None, :], (0, cfg.filter_length // 4), mode="reflect")
        ft = F.conv1d(xp, w["_model.stft.forward_basis_buffer"], stride=cfg.hop)
        nb = cfg.bins
        y = torch.sqrt(ft[:, :nb] ** 2 + ft[:, nb:] ** 2)
        for i, s in enumerate(cfg.enc_strides):
            p = f"_model.encoder.{i}.reparam_conv."
            y = F.relu(F.conv1d(y, w[p + "weight"], w[p + "bias"], stride=s, padding=1))
        return y[:, :, 0]

    def lstm(self, x, h, c):
        w = self.w
        g = (x @ w["_model.decoder.rnn.weight_ih"].t() + w["_model.decoder.rnn.bias_ih"]
             + h @ w["_model.decoder.rnn.weight_hh"].t() + w["_model.decoder.rnn.bias_hh"])
        i, f, gg, o = g.chunk(4, dim=-1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        return h, c

    def head(self, h):
        w = self.w
        v = F.relu(h) @ w["_model.decoder.decoder.2.weight"][0, :, 0] + w["_model.decoder.decoder.2.bias"][0]
        return torch.sigmoid(v)

    def window(self, x: np.ndarray, state: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        with torch.no_grad():
            xt = torch.from_numpy(np.asarray(x, np.float32))
            st = torch.from_numpy(np.asarray(state, np.float32))
            h, c = self.lstm(self.encode(xt), st[0], st[1])
            p = self.head(h)
            return p[:, None].numpy(), torch.stack([h, c]).numpy()

    def session(self):
        oracle = self

        class _Session:
            def run(self, output_names, feeds):
                return list(oracle.window(feeds["input"], feeds["state"]))
        return _Session()

    def probs_batched(self, audio: np.ndarray) -> np.ndarray:
        """run_windows with the encoder batched over all windows (same math, not bit-equal
        summation order); for larger cases."""
        n = len(audio) // WINDOW
        if n == 0:
            return np.zeros(0, np.float32)
        a = np.asarray(audio, np.float32)
        ctx = np.zeros((n, CONTEXT), np.float32)
        body = a[:n * WINDOW].reshape(n, WINDOW)
        ctx[1:] = body[:-1, -CONTEXT:]
        with torch.no_grad():
            enc = self.encode(torch.from_numpy(np.concatenate([ctx, body], 1)))
            h = torch.zeros(1, self.cfg.hidden)
            c = torch.zeros(1, self.cfg.hidden)
            out = np.empty(n, np.float32)
            for t in range(n):
                h, c = self.lstm(enc[t:t + 1], h, c)
                out[t] = float(self.head(h)[0])
        return out


def run_windows(session, audio: np.ndarray, sample_rate: int = 16000) -> np.ndarray:
    """Speech probability per 512-sample window (core/vad_utils.py:80-111)."""
    n = len(audio) // WINDOW
    state = np.zeros((2, 1, 128), np.float32)
    sr = np.array(sample_rate, np.int64)
    context = np.zeros(CONTEXT, np.float32)
    probs = []
    for i in range(n):
        chunk = audio[i * WINDOW:(i + 1) * WINDOW]
        x = np.concatenate([context, chunk]).reshape(1, -1).astype(np.float32)
        out, state = session.run(None, {"input": x, "state": state, "sr": sr})
        probs.append(float(out[0][0]))
        context = chunk[-CONTEXT:]
    return np.array(probs, np.float32)


def speech_windows(probs, threshold: float, min_silence_ms: int, min_speech_ms: int,
                   sample_rate: int = 16000) -> List[Tuple[int, int]]:
    """Window-index speech segments (core/vad_utils.py:120-151), literally."""
    min_sil = int(min_silence_ms * sample_rate / 1000 / WINDOW)
    min_sp = int(min_speech_ms * sample_rate / 1000 / WINDOW)
    segs, is_speech, start, sil = [], False, 0, 0
    for i, p in enumerate(probs):
        p = float(p)  # the reference compares Python floats (f64), :103, :130
        if p >= threshold:
            if not is_speech:
                start, is_speech = i, True
            sil = 0
        elif is_speech:
            sil += 1
            if sil >= min_sil:
                end = i - sil + 1
                if end - start >= min_sp:
                    segs.append((start, end))
                is_speech, sil = False, 0
    if is_speech and len(probs) - start >= min_sp:
        segs.append((start, len(probs)))
    return segs


def vad_segments(audio: np.ndarray, probs_fn, sample_rate: int = 16000, threshold: float = 0.2,
                 min_silence_ms: int = 100, min_speech_ms: int = 250, padding_ms: int = 1000,
                 merge_gap_ms: int = 250, auto_boost: bool = True, fallback_full: bool = True):
    """get_vad_segments (core/vad_utils.py:158-260); probs_fn(audio) -> per-window probs."""
    total = len(audio)
    if total < WINDOW:
        return [(0, total)] if fallback_full else []
    a = audio
    if auto_boost:
        m = np.max(np.abs(audio))
        if 1e-6 < m < 0.071:
            a = (audio * (0.071 / m)).astype(np.float32)
    probs = probs_fn(a)
    segs = speech_windows(probs, threshold, min_silence_ms, min_speech_ms, sample_rate)
    if not segs:
        segs = speech_windows(probs, 0.3, 100, 150, sample_rate)
    if not segs:
        return [(0, total)] if fallback_full else []
    pad = int(padding_ms * sample_rate / 1000)
    res = [(max(0, s * WINDOW - pad), min(total, e * WINDOW + pad)) for s, e in segs]
    if merge_gap_ms > 0 and len(res) > 1:
        gap = int(merge_gap_ms * sample_rate / 1000)
        merged = [res[0]]
        for s, e in res[1:]:
            if s - merged[-1][1] < gap:
                merged[-1] = (merged[-1][0], e)
            else:
                merged.append((s, e))
        res = merged
    return res
