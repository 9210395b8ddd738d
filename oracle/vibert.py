"""ORACLE (test infrastructure only) — ViBERT Seq2Labels forward, restated in torch fp32.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.

Restates the graph the reference runs with onnxruntime at core/gec_model.py:366-412: the
reference's convert_onnx/export_vibert_onnx.py Seq2LabelsModel.forward (:118-160) =
transformers BertModel (embeddings word + position + token type -> LayerNorm; per layer
self-attention with the additive padding mask, output dense + residual + LayerNorm,
intermediate dense + GELU (erf) + output dense + residual + LayerNorm), the sequence output
gathered at input_offsets, classifier and detector heads.  Pinned by
tests/golden/make_golden_vibert.py (the reference's own Seq2LabelsModel on seeded weights).
"""
from __future__ import annotations

import math
from typing import Dict, Tuple

import numpy as np
import torch
import torch.nn.functional as F


class VibertOracle:
    def __init__(self, cfg, weights: Dict[str, np.ndarray]):
        self.cfg = cfg
        self.w = {k: torch.from_numpy(np.asarray(v, np.float32)) for k, v in weights.items()}

    def _lin(self, x, name):
        return x @ self.w[name + ".weight"].t() + self.w[name + ".bias"]

    def _ln(self, x, name):
        return F.layer_norm(x, (x.shape[-1],), self.w[name + ".weight"], self.w[name + ".bias"],
                            self.cfg.layer_norm_eps)

    def run(self, input_ids, attention_mask, token_type_ids, input_offsets
            ) -> Tuple[np.ndarray, np.ndarray]:
        cfg, w = self.cfg, self.w
        with torch.no_grad():
            ids = torch.from_numpy(np.asarray(input_ids, np.int64))
            tt = torch.from_numpy(np.asarray(token_type_ids, np.int64))
            am = torch.from_numpy(np.asarray(attention_mask, np.int64))
            off = torch.from_numpy(np.asarray(input_offsets, np.int64))
            B, L = ids.shape
            pos = torch.arange(L)
            x = (w["bert.embeddings.word_embeddings.weight"][ids]
                 + w["bert.embeddings.position_embeddings.weight"][pos][None]
                 + w["bert.embeddings.token_type_embeddings.weight"][tt])
            x = self._ln(x, "bert.embeddings.LayerNorm")
            nh = cfg.num_attention_heads
            hd = cfg.hidden_size // nh
            bias = (1.0 - am[:, None, None, :].float()) * torch.finfo(torch.float32).min
            for i in range(cfg.num_hidden_layers):
                p = f"bert.encoder.layer.{i}."
                q = self._lin(x, p + "attention.self.query").view(B, L, nh, hd).transpose(1, 2)
                k = self._lin(x, p + "attention.self.key").view(B, L, nh, hd).transpose(1, 2)
                v = self._lin(x, p + "attention.self.value").view(B, L, nh, hd).transpose(1, 2)
                s = q @ k.transpose(-1, -2) / math.sqrt(hd) + bias
                ctx = (torch.softmax(s, dim=-1) @ v).transpose(1, 2).reshape(B, L, -1)
                x = self._ln(self._lin(ctx, p + "attention.output.dense") + x,
                             p + "attention.output.LayerNorm")
                h = F.gelu(self._lin(x, p + "intermediate.dense"))
                x = self._ln(self._lin(h, p + "output.dense") + x, p + "output.LayerNorm")
            g = x[torch.arange(B)[:, None], off]
            return (self._lin(g, "classifier").numpy().astype(np.float32),
                    self._lin(g, "detector").numpy().astype(np.float32))
