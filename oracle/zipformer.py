"""ORACLE (test infrastructure only) — torch fp32 restatement of the Zipformer2 transducer.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module; the product path (sherpa-vietnamese-asr_amd/) never does.

What it restates: the encoder / decoder / joiner graphs that the reference runs through
onnxruntime at `core/asr_engine.py:1045-1049` (encoder), `:1051-1056,1083-1088` (decoder)
and `:1090-1093` (joiner).  The graphs themselves are NOT in /root/reference (only the
absent .onnx files hold them), so this follows icefall's `zipformer/{zipformer,scaling,
subsampling,decoder,joiner,export-onnx}.py` (3P, unpinned by the reference) in inference
mode: Balancer/Whiten/Dropout are identities, bypass scales are used unclamped, the
exported encoder includes `encoder_proj`, the exported decoder includes `decoder_proj`.

Parity status: PARITY UNPINNED against the real ONNX graphs (weights and graphs are
absent offline).  Batch is always 1, exactly like the reference
(`core/asr_engine.py:1045-1046`), so the HIP path's batched/ragged execution is checked
against true per-sequence semantics.

Layout follows icefall: activations are (time, batch, channels).
"""
from __future__ import annotations

import math
import sys
import os
from typing import Dict, Tuple

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "sherpa-vietnamese-asr_amd"))
from zasr.model import ZipformerConfig, stack_prefix  # noqa: E402


def swoosh_l(x):
    # SwooshL(x) = log(1 + exp(x - 4)) - 0.08 x - 0.035   (icefall scaling.py SwooshLOnnx)
    return torch.nn.functional.softplus(x - 4.0) - 0.08 * x - 0.035


def swoosh_r(x):
    # SwooshR(x) = log(1 + exp(x - 1)) - 0.08 x - 0.313261687
    return torch.nn.functional.softplus(x - 1.0) - 0.08 * x - 0.313261687


def bias_norm(x, bias, log_scale):
    # BiasNorm: x * exp(log_scale) / sqrt(mean((x - bias)^2)) over channels
    scales = torch.mean((x - bias) ** 2, dim=-1, keepdim=True) ** -0.5 * torch.exp(log_scale)
    return x * scales


def compact_rel_pos_emb(T: int, pos_dim: int) -> torch.Tensor:
    """CompactRelPositionalEncoding rows for relative offsets x = -(T-1) .. (T-1)."""
    x = torch.arange(-(T - 1), T, dtype=torch.float32).unsqueeze(1)
    freqs = 1 + torch.arange(pos_dim // 2, dtype=torch.float32)
    compression_length = pos_dim ** 0.5
    x_compressed = (compression_length * x.sign()
                    * ((x.abs() + compression_length).log() - math.log(compression_length)))
    length_scale = pos_dim / (2.0 * math.pi)
    x_atan = (x_compressed / length_scale).atan()
    pe = torch.zeros(x.shape[0], pos_dim)
    pe[:, 0::2] = (x_atan * freqs).cos()
    pe[:, 1::2] = (x_atan * freqs).sin()
    pe[:, -1] = 1.0
    return pe  # (2T-1, pos_dim)


class ZipformerOracle:
    """Batch-1 fp32 forward of encoder (incl. encoder_proj), decoder and joiner."""

    def __init__(self, cfg: ZipformerConfig, weights: Dict[str, np.ndarray]):
        self.cfg = cfg
        self.w = {k: torch.from_numpy(np.asarray(v, dtype=np.float32)) for k, v in weights.items()}

    # ---------------- encoder_embed (Conv2dSubsampling) ----------------
    def _lin(self, x, name, bias=True):
        y = x @ self.w[name + ".weight"].t()
        return y + self.w[name + ".bias"] if bias else y

    def encoder_embed(self, feats: torch.Tensor) -> torch.Tensor:
        """feats (T, 80) -> (L, d0); L = (T - 7) // 2."""
        F = torch.nn.functional
        w = self.w
        x = feats.unsqueeze(0).unsqueeze(0)  # (1, 1, T, 80)
        x = swoosh_r(F.conv2d(x, w["encoder_embed.conv.0.weight"], w["encoder_embed.conv.0.bias"],
                              padding=(0, 1)))
        x = swoosh_r(F.conv2d(x, w["encoder_embed.conv.4.weight"], w["encoder_embed.conv.4.bias"],
                              stride=2))
        x = swoosh_r(F.conv2d(x, w["encoder_embed.conv.7.weight"], w["encoder_embed.conv.7.bias"],
                              stride=(1, 2)))
        # ConvNeXt(128), kernel (7, 7)
        c = x.shape[1]
        y = F.conv2d(x, w["encoder_embed.convnext.depthwise_conv.weight"],
                     w["encoder_embed.convnext.depthwise_conv.bias"], padding=(3, 3), groups=c)
        y = F.conv2d(y, w["encoder_embed.convnext.pointwise_conv1.weight"],
                     w["encoder_embed.convnext.pointwise_conv1.bias"])
        y = swoosh_l(y)
        y = F.conv2d(y, w["encoder_embed.convnext.pointwise_conv2.weight"],
                     w["encoder_embed.convnext.pointwise_conv2.bias"])
        x = x + y
        b, c, t, f = x.shape
        x = x.transpose(1, 2).reshape(b, t, c * f)
        x = self._lin(x, "encoder_embed.out")
        x = bias_norm(x, w["encoder_embed.out_norm.bias"], w["encoder_embed.out_norm.log_scale"])
        return x[0]

    # ---------------- Zipformer2 encoder layer ----------------
    def _attn_weights(self, P, x, pos_emb, h):
        cfg = self.cfg
        qd, pd = cfg.query_head_dim, cfg.pos_head_dim
        T = x.shape[0]
        x = self._lin(x, P + "self_attn_weights.in_proj")
        q = x[..., 0:qd * h].reshape(T, 1, h, qd).permute(2, 1, 0, 3)
        k = x[..., qd * h:2 * qd * h].reshape(T, 1, h, qd).permute(2, 1, 3, 0)
        p = x[..., 2 * qd * h:].reshape(T, 1, h, pd).permute(2, 1, 0, 3)
        attn_scores = torch.matmul(q, k)  # (h, 1, T, T)
        pe = pos_emb @ self.w[P + "self_attn_weights.linear_pos.weight"].t()  # (2T-1, h*pd)
        pe = pe.reshape(1, 2 * T - 1, h, pd).permute(2, 0, 3, 1)  # (h, 1, pd, 2T-1)
        pos_scores = torch.matmul(p, pe)  # (h, 1, T, 2T-1)
        # relative -> absolute: column n = (T-1) - i + j  (icefall's as_strided form)
        pos_scores = pos_scores.as_strided(
            (h, 1, T, T),
            (pos_scores.stride(0), pos_scores.stride(1),
             pos_scores.stride(2) - pos_scores.stride(3), pos_scores.stride(3)),
            storage_offset=pos_scores.stride(3) * (T - 1))
        attn_scores = attn_scores + pos_scores
        return torch.softmax(attn_scores, dim=-1)  # (h, 1, T, T)

    def _ff(self, name, x):
        return self._lin(swoosh_l(self._lin(x, name + ".in_proj")), name + ".out_proj")

    def _self_attn(self, name, x, attn_weights):
        T = x.shape[0]
        h = attn_weights.shape[0]
        v = self._lin(x, name + ".in_proj").reshape(T, 1, h, -1).permute(2, 1, 0, 3)
        y = torch.matmul(attn_weights, v).permute(2, 1, 0, 3).reshape(T, 1, -1)
        return self._lin(y, name + ".out_proj")

    def _nonlin_attn(self, name, x, attn_weights0):
        T = x.shape[0]
        x = self._lin(x, name + ".in_proj")
        s, x, y = x.chunk(3, dim=2)
        x = x * torch.tanh(s)
        x = x.reshape(T, 1, 1, -1).permute(2, 1, 0, 3)
        x = torch.matmul(attn_weights0, x).permute(2, 1, 0, 3).reshape(T, 1, -1)
        x = x * y
        return self._lin(x, name + ".out_proj")

    def _conv_module(self, name, x):
        F = torch.nn.functional
        x = self._lin(x, name + ".in_proj")
        x, s = x.chunk(2, dim=2)
        x = x * torch.sigmoid(s)
        x = x.permute(1, 2, 0)  # (1, C, T)
        wdw = self.w[name + ".depthwise_conv.weight"]
        x = F.conv1d(x, wdw, self.w[name + ".depthwise_conv.bias"],
                     padding=wdw.shape[-1] // 2, groups=wdw.shape[0])
        x = x.permute(2, 0, 1)
        return self._lin(swoosh_r(x), name + ".out_proj")

    def _layer(self, P, src, pos_emb, h):
        w = self.w
        src_orig = src
        attn_weights = self._attn_weights(P, src, pos_emb, h)
        src = src + self._ff(P + "feed_forward1", src)
        src = src + self._nonlin_attn(P + "nonlin_attention", src, attn_weights[0:1])
        src = src + self._self_attn(P + "self_attn1", src, attn_weights)
        src = src + self._conv_module(P + "conv_module1", src)
        src = src + self._ff(P + "feed_forward2", src)
        src = src_orig + (src - src_orig) * w[P + "bypass_mid.bypass_scale"]
        src = src + self._self_attn(P + "self_attn2", src, attn_weights)
        src = src + self._conv_module(P + "conv_module2", src)
        src = src + self._ff(P + "feed_forward3", src)
        src = bias_norm(src, w[P + "norm.bias"], w[P + "norm.log_scale"])
        src = src_orig + (src - src_orig) * w[P + "bypass.bypass_scale"]
        return src

    @staticmethod
    def _downsample(src, bias):
        T = src.shape[0]
        ds = bias.shape[0]
        dT = (T + ds - 1) // ds
        pad = dT * ds - T
        src = torch.cat((src, src[T - 1:].expand(pad, src.shape[1], src.shape[2])), dim=0)
        src = src.reshape(dT, ds, src.shape[1], src.shape[2])
        wts = bias.softmax(dim=0).unsqueeze(-1).unsqueeze(-1)
        return (src * wts).sum(dim=1)

    def encoder(self, feats: np.ndarray, return_stacks: bool = False):
        """feats (T, 80) float32 -> encoder_out (T', joiner_dim)."""
        cfg, w = self.cfg, self.w
        with torch.no_grad():
            x = self.encoder_embed(torch.from_numpy(np.asarray(feats, dtype=np.float32)))
            x = x.unsqueeze(1)  # (L, 1, d0)
            outputs = []
            for i in range(cfg.num_stacks):
                d, ds = cfg.encoder_dims[i], cfg.downsampling[i]
                if d <= x.shape[-1]:
                    x = x[..., :d]
                else:
                    x = torch.cat((x, torch.zeros(x.shape[0], x.shape[1], d - x.shape[-1])), dim=-1)
                pre = stack_prefix(i, cfg)
                src_orig = x
                if ds != 1:
                    x = self._downsample(x, w[f"encoder.encoders.{i}.downsample.bias"])
                pos_emb = compact_rel_pos_emb(x.shape[0], cfg.pos_dim)
                for j in range(cfg.num_layers[i]):
                    x = self._layer(f"{pre}layers.{j}.", x, pos_emb, cfg.num_heads[i])
                if ds != 1:
                    x = x.unsqueeze(1).expand(x.shape[0], ds, 1, d).reshape(x.shape[0] * ds, 1, d)
                    x = x[: src_orig.shape[0]]
                    s = w[f"encoder.encoders.{i}.out_combiner.bypass_scale"]
                    x = src_orig + (x - src_orig) * s
                outputs.append(x)
            # full-dim output: each channel from the most recent stack that has it
            pieces = [outputs[-1]]
            cur = cfg.encoder_dims[-1]
            for i in range(cfg.num_stacks - 2, -1, -1):
                d = cfg.encoder_dims[i]
                if d > cur:
                    pieces.append(outputs[i][..., cur:d])
                    cur = d
            x = torch.cat(pieces, dim=-1)
            x = self._downsample(x, w["encoder.downsample_output.bias"])
            x = self._lin(x[:, 0, :], "encoder_proj")
        out = x.numpy().astype(np.float32)
        if return_stacks:
            return out, [o[:, 0, :].numpy() for o in outputs]
        return out

    # ---------------- decoder / joiner ----------------
    def decoder(self, y: np.ndarray) -> np.ndarray:
        """y int64 (B, context_size), already clamped >= 0 (core/asr_engine.py:1052,1075)."""
        F = torch.nn.functional
        w = self.w
        with torch.no_grad():
            yt = torch.from_numpy(np.asarray(y, dtype=np.int64))
            emb = w["decoder.embedding.weight"][yt.clamp(min=0)] * (yt >= 0).unsqueeze(-1)
            emb = emb.permute(0, 2, 1)  # (B, D, ctx)
            D = emb.shape[1]
            out = F.conv1d(emb, w["decoder.conv.weight"], None, groups=D // 4).permute(0, 2, 1)
            out = F.relu(out)[:, 0, :]
            out = out @ w["decoder_proj.weight"].t() + w["decoder_proj.bias"]
        return out.numpy().astype(np.float32)

    def joiner(self, enc: np.ndarray, dec: np.ndarray) -> np.ndarray:
        w = self.w
        with torch.no_grad():
            x = torch.tanh(torch.from_numpy(enc) + torch.from_numpy(dec))
            out = x @ w["joiner.output_linear.weight"].t() + w["joiner.output_linear.bias"]
        return out.numpy().astype(np.float32)
