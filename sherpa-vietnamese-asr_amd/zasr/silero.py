"""Silero VAD (16 kHz) model description, synthetic weights and on-disk format (SURVEY §8f
row 4).

The reference runs models/silero-vad/silero_vad_16k_op15.onnx (snakers4/silero-vad master,
sha256 7ed98ddb..., build-portable/prepare_offline_build.py:211-219) with onnxruntime, one
512-sample window at a time with 64 samples of left context and the (2, 1, 128) LSTM state
carried between calls (core/vad_utils.py:62-111).  The network is silero-vad v5's 16 kHz
branch (third-party; neither the .onnx nor the silero_vad package ships with the reference or
this image), restated from its published architecture:

  input [N, 576] (64 context + 512 window)
  STFT:     ReflectionPad1d((0, 64)) -> Conv1d(1 -> 258, k 256, stride 128, basis buffer)
            -> magnitude sqrt(re^2 + im^2) of the 129 bins -> [N, 129, 4]
  encoder:  4 x (Conv1d(k 3, pad 1) + ReLU): 129->128 s1, 128->64 s2, 64->64 s2, 64->128 s1
            -> [N, 128, 1]
  decoder:  LSTMCell(128, 128) on the carried (h, c); ReLU; Conv1d(128 -> 1, k 1); sigmoid
  output    speech probability [N, 1], new state stack(h, c) [2, N, 128]

Weights are SYNTHETIC (seeded numpy PCG64) under the torch state-dict names of the 16 kHz
model ("_model." prefix); the STFT basis is the real-DFT basis with a periodic Hann window, as
in silero's STFT module, and the other layers are scaled so the speech probability follows the
signal's energy envelope (so VAD segmentation is exercised on synthetic speech).
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np

WINDOW = 512          # core/vad_utils.py:81
CONTEXT = 64          # :82
SR = 16000


@dataclasses.dataclass
class SileroConfig:
    sample_rate: int = SR
    window: int = WINDOW
    context: int = CONTEXT
    filter_length: int = 256
    hop: int = 128
    enc_channels: Tuple[int, ...] = (128, 64, 64, 128)
    enc_strides: Tuple[int, ...] = (1, 2, 2, 1)
    hidden: int = 128

    @property
    def bins(self) -> int:
        return self.filter_length // 2 + 1

    @property
    def stft_frames(self) -> int:
        padded = self.context + self.window + self.filter_length // 4
        return (padded - self.filter_length) // self.hop + 1

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=1)

    @staticmethod
    def from_json(text: str) -> "SileroConfig":
        d = json.loads(text)
        d["enc_channels"] = tuple(d["enc_channels"])
        d["enc_strides"] = tuple(d["enc_strides"])
        return SileroConfig(**d)


P = "_model."


def param_shapes(cfg: SileroConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    s[P + "stft.forward_basis_buffer"] = (2 * cfg.bins, 1, cfg.filter_length)
    cin = cfg.bins
    for i, co in enumerate(cfg.enc_channels):
        s[P + f"encoder.{i}.reparam_conv.weight"] = (co, cin, 3)
        s[P + f"encoder.{i}.reparam_conv.bias"] = (co,)
        cin = co
    H = cfg.hidden
    s[P + "decoder.rnn.weight_ih"] = (4 * H, cin)
    s[P + "decoder.rnn.weight_hh"] = (4 * H, H)
    s[P + "decoder.rnn.bias_ih"] = (4 * H,)
    s[P + "decoder.rnn.bias_hh"] = (4 * H,)
    s[P + "decoder.decoder.2.weight"] = (1, H, 1)
    s[P + "decoder.decoder.2.bias"] = (1,)
    return s


def stft_basis(cfg: SileroConfig) -> np.ndarray:
    n = cfg.filter_length
    k = np.arange(cfg.bins)[:, None]
    t = np.arange(n)[None, :]
    win = 0.5 - 0.5 * np.cos(2 * np.pi * np.arange(n) / n)      # periodic Hann
    ang = 2 * np.pi * k * t / n
    basis = np.concatenate([np.cos(ang), -np.sin(ang)], 0) * win[None, :]
    return basis[:, None, :].astype(np.float32)


def synth_weights(cfg: SileroConfig, seed: int = 20261019) -> Dict[str, np.ndarray]:
    """Seeded weights. Encoder convs are mostly positive (magnitude features stay
    informative), the LSTM has a moderate recurrent gain, and the decoder maps the hidden
    state to a probability that rises with input energy."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out: Dict[str, np.ndarray] = {}
    for name, shape in param_shapes(cfg).items():
        if name.endswith("forward_basis_buffer"):
            w = stft_basis(cfg)
        elif ".encoder." in name and name.endswith("weight"):
            fan = shape[1] * shape[2]
            w = rng.normal(0.5, 1.0, size=shape) / math.sqrt(fan)
            if name.startswith(P + "encoder.0."):
                w = w * 4.0   # |STFT| of speech-level audio is O(0.1-1)
        elif ".encoder." in name:
            w = rng.normal(-0.05, 0.05, size=shape)
        elif name.endswith("weight_ih"):
            w = rng.normal(0.0, 1.0, size=shape) / math.sqrt(shape[1])
            w[2 * cfg.hidden:3 * cfg.hidden] += 0.25 / math.sqrt(shape[1])
        elif name.endswith("weight_hh"):
            w = rng.normal(0.0, 0.8, size=shape) / math.sqrt(shape[1])
        elif name.endswith("bias_ih") or name.endswith("bias_hh"):
            w = rng.normal(0.0, 0.1, size=shape)
        elif name.endswith("decoder.2.weight"):
            w = np.abs(rng.normal(0.0, 1.0, size=shape)) * (6.0 / math.sqrt(shape[1]))
        else:  # decoder.2.bias
            w = np.full(shape, -5.0)
        out[name] = np.ascontiguousarray(w, dtype=np.float32)
    return out


def save_model_dir(path: str, cfg: SileroConfig, weights: Dict[str, np.ndarray]) -> str:
    """silero_config.json + silero_vad.safetensors (the engine's Silero VAD format)."""
    from safetensors.numpy import save_file
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "silero_config.json"), "w") as f:
        f.write(cfg.to_json())
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()},
              os.path.join(path, "silero_vad.safetensors"))
    return path


def window_flops(cfg: SileroConfig) -> float:
    """Multiply-adds x 2 of one 512-sample window (STFT conv + encoder + LSTM + decoder)."""
    T = cfg.stft_frames
    f = 2.0 * T * 2 * cfg.bins * cfg.filter_length
    cin, t = cfg.bins, T
    for co, s in zip(cfg.enc_channels, cfg.enc_strides):
        t = (t + 2 - 3) // s + 1
        f += 2.0 * t * co * cin * 3
        cin = co
    H = cfg.hidden
    f += 2.0 * 4 * H * (cin + H) + 2.0 * H
    return f
