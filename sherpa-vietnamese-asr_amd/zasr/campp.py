"""CAM++ speaker-embedding model description, synthetic weights, on-disk
format and the embedding-window plan.

The reference runs the 3D-Speaker CAM++ export (campplus_cn_en_common_200k.onnx, 192-dim)
through onnxruntime on batches of 1.5 s fbank windows (core/speaker_diarization_senko_campp_
optimized.py:519-620); the architecture is the reference's own
convert_onnx/export_campplus_onnx.py:17-270 (CAMPPlus(feat_dim=80, embedding_size=192,
growth_rate=32, bn_size=4, init_channels=128, config_str="batchnorm-relu")).  This module
restates its parameter set under the same state-dict names so that a checkpoint or an ONNX
export maps by name.

Weights in this repo are always SYNTHETIC (seeded numpy PCG64): no checkpoint is available
offline.  BatchNorm running statistics are random too (eval-mode BN is an affine map).
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

SR = 16000
BN_EPS = 1e-5


@dataclasses.dataclass
class CamppConfig:
    feat_dim: int = 80
    embedding_size: int = 192
    growth_rate: int = 32
    bn_size: int = 4
    init_channels: int = 128
    m_channels: int = 32          # FCM head channels
    head_blocks: Tuple[int, ...] = (2, 2)
    block_layers: Tuple[int, ...] = (12, 24, 16)
    block_kernels: Tuple[int, ...] = (3, 3, 3)
    block_dilations: Tuple[int, ...] = (1, 2, 2)
    seg_len: int = 100            # CAMLayer.seg_pooling segment (frames)

    @property
    def bn_channels(self) -> int:
        return self.bn_size * self.growth_rate

    @property
    def head_out(self) -> int:
        return self.m_channels * (self.feat_dim // 8)

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=1)

    @staticmethod
    def from_json(text: str) -> "CamppConfig":
        d = json.loads(text)
        for k, v in list(d.items()):
            if isinstance(v, list):
                d[k] = tuple(v)
        return CamppConfig(**d)


def _bn(s, name, c, affine=True):
    if affine:
        s[name + ".weight"] = (c,)
        s[name + ".bias"] = (c,)
    s[name + ".running_mean"] = (c,)
    s[name + ".running_var"] = (c,)


def param_shapes(cfg: CamppConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    """State-dict names / shapes of CAMPPlus (num_batches_tracked buffers omitted)."""
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    m = cfg.m_channels
    s["head.conv1.weight"] = (m, 1, 3, 3)
    _bn(s, "head.bn1", m)
    for li, nb in enumerate(cfg.head_blocks):
        for b in range(nb):
            p = f"head.layer{li + 1}.{b}."
            s[p + "conv1.weight"] = (m, m, 3, 3)
            _bn(s, p + "bn1", m)
            s[p + "conv2.weight"] = (m, m, 3, 3)
            _bn(s, p + "bn2", m)
            if b == 0:  # stride (2, 1): projection shortcut
                s[p + "shortcut.0.weight"] = (m, m, 1, 1)
                _bn(s, p + "shortcut.1", m)
    s["head.conv2.weight"] = (m, m, 3, 3)
    _bn(s, "head.bn2", m)
    c = cfg.init_channels
    s["xvector.tdnn.linear.weight"] = (c, cfg.head_out, 5)
    _bn(s, "xvector.tdnn.nonlinear.batchnorm", c)
    g, bnc = cfg.growth_rate, cfg.bn_channels
    for bi, (nl, k) in enumerate(zip(cfg.block_layers, cfg.block_kernels)):
        for i in range(nl):
            p = f"xvector.block{bi + 1}.tdnnd{i + 1}."
            cin = c + i * g
            _bn(s, p + "nonlinear1.batchnorm", cin)
            s[p + "linear1.weight"] = (bnc, cin, 1)
            _bn(s, p + "nonlinear2.batchnorm", bnc)
            s[p + "cam_layer.linear_local.weight"] = (g, bnc, k)
            s[p + "cam_layer.linear1.weight"] = (bnc // 2, bnc, 1)
            s[p + "cam_layer.linear1.bias"] = (bnc // 2,)
            s[p + "cam_layer.linear2.weight"] = (g, bnc // 2, 1)
            s[p + "cam_layer.linear2.bias"] = (g,)
        c = c + nl * g
        _bn(s, f"xvector.transit{bi + 1}.nonlinear.batchnorm", c)
        s[f"xvector.transit{bi + 1}.linear.weight"] = (c // 2, c, 1)
        c //= 2
    _bn(s, "xvector.out_nonlinear.batchnorm", c)
    s["xvector.dense.linear.weight"] = (cfg.embedding_size, 2 * c, 1)
    _bn(s, "xvector.dense.nonlinear.batchnorm", cfg.embedding_size, affine=False)
    return s


def synth_weights(cfg: CamppConfig, seed: int = 20261017) -> Dict[str, np.ndarray]:
    """Seeded synthetic weights: convs ~ N(0, 2 / fan_in) (kaiming, as CAMPPlus.__init__),
    BN affine near identity, running statistics random (mean ~ N(0, 0.1), var ~ U(0.5, 1.5))."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in param_shapes(cfg).items():
        if name.endswith("running_mean"):
            w = rng.normal(0.0, 0.1, size=shape)
        elif name.endswith("running_var"):
            w = rng.uniform(0.5, 1.5, size=shape)
        elif ("bn" in name.split(".")[-2] or "batchnorm" in name or "shortcut.1" in name) \
                and name.endswith(".weight"):
            w = rng.uniform(0.8, 1.2, size=shape)
        elif name.endswith(".bias"):
            w = rng.normal(0.0, 0.05, size=shape)
        else:
            fan_in = int(np.prod(shape[1:]))
            w = rng.normal(0.0, math.sqrt(2.0 / fan_in), size=shape)
        out[name] = np.ascontiguousarray(w, dtype=np.float32)
    return out


def save_model_dir(path: str, cfg: CamppConfig, weights: Dict[str, np.ndarray]) -> str:
    """campp_config.json + campp.safetensors (the engine's CAM++ format; a reference
    campplus_cn_en_common_200k.onnx next to them maps by the same names)."""
    from safetensors.numpy import save_file
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "campp_config.json"), "w") as f:
        f.write(cfg.to_json())
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()},
              os.path.join(path, "campp.safetensors"))
    return path


def window_plan(n_region_frames: int, window_frames: int = 150, step_frames: int = 60
                ) -> List[Tuple[int, int]]:
    """[(first frame, frame count)] of the embedding windows of one speech region's fbank
    (core/speaker_diarization_senko_campp_optimized.py:561-582): a region shorter than a window
    is one window of all its frames; otherwise windows every `step_frames` while
    pos + window < n (strict), then a tail window pulled back to end at the region's end."""
    if n_region_frames < 10:
        return []
    if n_region_frames < window_frames:
        return [(0, n_region_frames)]
    out = []
    pos = 0
    while pos + window_frames < n_region_frames:
        out.append((pos, window_frames))
        pos += step_frames
    out.append((max(0, n_region_frames - window_frames), window_frames))
    return out


def campp_flops(cfg: CamppConfig, T: int) -> float:
    """Algorithmic FLOPs of one window of T fbank frames (convolutions / projections)."""
    m, F = cfg.m_channels, cfg.feat_dim
    fl = 2.0 * 9 * m * F * T  # conv1 (1 -> m) at F x T
    f = F
    for nb in cfg.head_blocks:
        f2 = (f + 1) // 2
        fl += 2.0 * 9 * m * m * f2 * T + 2.0 * m * m * f2 * T  # strided conv1 + shortcut
        fl += 2.0 * 9 * m * m * f2 * T                          # conv2
        fl += (nb - 1) * 2 * 2.0 * 9 * m * m * f2 * T           # remaining blocks
        f = f2
    f2 = (f + 1) // 2
    fl += 2.0 * 9 * m * m * f2 * T
    T2 = (T - 1) // 2 + 1
    c = cfg.init_channels
    fl += 2.0 * 5 * cfg.head_out * c * T2
    g, bnc = cfg.growth_rate, cfg.bn_channels
    for nl, k in zip(cfg.block_layers, cfg.block_kernels):
        for i in range(nl):
            cin = c + i * g
            fl += 2.0 * cin * bnc * T2 + 2.0 * k * bnc * g * T2
        c += nl * g
        fl += 2.0 * c * (c // 2) * T2
        c //= 2
    fl += 2.0 * 2 * c * cfg.embedding_size
    return fl
