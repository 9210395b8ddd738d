"""Precision-mode simulation on the CPU (development tool, test infrastructure: imports the
oracle).  Runs the 68M oracle with every contraction (linear layers, the frontend convs,
q.k, p.pe, attention @ v, the NonlinAttention product, the joiner) emulated at a reduced
operand precision and reports the token error rate of greedy / beam 8 + hotwords against the
plain fp32 oracle on tests/test_gpu_e2e.py's three chunks -- the number the HIP modes are
measured by (test_m_bf16_token_error_rate).

Operand modes (f32 accumulate throughout):
  bf16   each operand rounded to bf16 (one MFMA)
  x3     hi + lo split of both operands, hi*hi + hi*lo + lo*hi (three bf16 MFMAs)
  x6     hi + mid + lo split, the six products down to 2^-24 (six bf16 MFMAs)
  h3     fp16 hi + lo with the lo piece scaled by 2^11, hi*hi + (hi*lo + lo*hi) * 2^-11
         (three fp16 MFMAs, ~2^-22 relative; operands must stay below 65504)

    python tests/precision_sim.py [modes...] [--joiner-f32]
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "sherpa-vietnamese-asr_amd")]

from oracle.zipformer import ZipformerOracle  # noqa: E402

_MODE = {"m": None}


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


def split(x, n):
    parts, r = [], x
    for _ in range(n):
        h = _bf(r)
        parts.append(h)
        r = r - h
    return parts


_RANGE = {"max": 0.0}


def _h(x):
    return x.to(torch.float16).to(torch.float32)


def hsplit(x):
    """fp16 hi + lo split with the lo piece pre-scaled by 2^11 (kept in the fp16 normal
    range): x = hi + lo * 2^-11 to ~2^-22 relative (the "fp16x3" operand format)."""
    _RANGE["max"] = max(_RANGE["max"], float(x.abs().max()) if x.numel() else 0.0)
    h = _h(x)
    return h, _h((x - h) * 2048.0)


def emu_mm(a, b):
    m = _MODE["m"]
    if m is None:
        return torch.matmul(a, b)
    if m == "h3":
        ah, al = hsplit(a)
        bh, bl = hsplit(b)
        return torch.matmul(ah, bh) + (torch.matmul(ah, bl) + torch.matmul(al, bh)) * (1.0 / 2048.0)
    if m == "bf16":
        return torch.matmul(_bf(a), _bf(b))
    if m == "x3":
        ah, al = split(a, 2)
        bh, bl = split(b, 2)
        return torch.matmul(ah, bh) + (torch.matmul(ah, bl) + torch.matmul(al, bh))
    if m == "x6":
        a0, a1, a2 = split(a, 3)
        b0, b1, b2 = split(b, 3)
        return (torch.matmul(a0, b0) + (torch.matmul(a0, b1) + torch.matmul(a1, b0))
                + (torch.matmul(a0, b2) + torch.matmul(a1, b1) + torch.matmul(a2, b0)))
    raise ValueError(m)


class SimOracle(ZipformerOracle):
    """ZipformerOracle with its contractions routed through emu_mm."""

    def _lin(self, x, name, bias=True):
        y = emu_mm(x, self.w[name + ".weight"].t())
        return y + self.w[name + ".bias"] if bias else y


_orig_matmul = torch.matmul


def run(modes, joiner_f32=False):
    from model_fixtures import m_model
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from test_gpu_e2e import M_SECS, _hotword_phrases, _speech, edit_distance

    cfg, w, _ = m_model()
    ref = ZipformerOracle(cfg, w)
    chunks = [_speech(s, 1200 + i) for i, s in enumerate(M_SECS)]
    feats = [fbank(c) for c in chunks]
    encs = [ref.encoder(f) for f in feats]
    greedy = [beam_search(e, ref.decoder, ref.joiner, 1) for e in encs]
    phrases, scores = _hotword_phrases(cfg.vocab_size, greedy[0][0])
    graph = HotwordGraph(phrases, scores)
    beam8 = [beam_search(e, ref.decoder, ref.joiner, 8, graph) for e in encs]
    out = {}
    sim = SimOracle(cfg, w)
    for m in modes:
        _MODE["m"] = m
        # attention / nonlin products go through torch.matmul, the frontend's dense convs
        # (conv.4, conv.7, the ConvNeXt pointwise pair) through F.conv2d inside the oracle
        torch.matmul = _route
        torch.nn.functional.conv2d = _conv
        try:
            se = [sim.encoder(f) for f in feats]
        finally:
            torch.matmul = _orig_matmul
            torch.nn.functional.conv2d = _orig_conv
        jo = ref.joiner if joiner_f32 else _sim_joiner(sim, m)
        rep = {}
        for name, beam, refr in (("greedy", 1, greedy), ("beam8_hotwords", 8, beam8)):
            res = [beam_search(e, ref.decoder, jo, beam, graph if beam > 1 else None) for e in se]
            errs = [edit_distance(r[0], g[0]) for r, g in zip(res, refr)]
            n = [len(g[0]) for g in refr]
            rep[name] = {"ter": round(sum(errs) / max(1, sum(n)), 5), "errs": errs, "ref_tokens": n}
        d = max(float(np.abs(a - b).max()) for a, b in zip(se, encs))
        out[m] = {"enc_max_abs_diff": d, **rep}
        if m == "h3":
            out[m]["max_abs_operand"] = _RANGE["max"]
        print(m, json.dumps(out[m]), flush=True)
    return out


_ATTN_F32 = {"on": False}


def _route(a, b):
    torch.matmul = _orig_matmul
    try:
        if _ATTN_F32["on"]:  # the HIP bf16x3 mode keeps the attention products in f32
            return torch.matmul(a, b)
        return emu_mm(a, b)
    finally:
        torch.matmul = _route


_orig_conv = torch.nn.functional.conv2d


def _conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    """Dense convs (groups == 1, more than one input channel: the GEMM-lowered ones) at the
    mode's operand precision; conv.0 (1 input channel) and the depthwise conv stay f32."""
    m = _MODE["m"]
    c = lambda u, v, bb=None: _orig_conv(u, v, bb, stride, padding, dilation, groups)
    if m is None or groups != 1 or x.shape[1] == 1:
        return c(x, w, b)
    if m == "bf16":
        return c(_bf(x), _bf(w), b)
    if m == "h3":
        xh, xl = hsplit(x)
        wh, wl = hsplit(w)
        return c(xh, wh, b) + (c(xh, wl) + c(xl, wh)) * (1.0 / 2048.0)
    if m == "x3":
        xh, xl = split(x, 2)
        wh, wl = split(w, 2)
        return c(xh, wh, b) + (c(xh, wl) + c(xl, wh))
    x0, x1, x2 = split(x, 3)
    w0, w1, w2 = split(w, 3)
    return c(x0, w0, b) + (c(x0, w1) + c(x1, w0)) + (c(x0, w2) + c(x1, w1) + c(x2, w0))


def _sim_joiner(sim, m):
    def j(enc, dec):
        _MODE["m"] = m
        with torch.no_grad():
            x = torch.tanh(torch.from_numpy(enc) + torch.from_numpy(dec))
            out = emu_mm(x, sim.w["joiner.output_linear.weight"].t()) + sim.w["joiner.output_linear.bias"]
        return out.numpy().astype(np.float32)
    return j


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    _ATTN_F32["on"] = "--attn-f32" in sys.argv
    res = run(args or ["bf16", "x3", "x6"], joiner_f32="--joiner-f32" in sys.argv)
    print(json.dumps(res, indent=1))
