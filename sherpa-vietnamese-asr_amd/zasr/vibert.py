"""ViBERT-capu punctuation / capitalization model description, synthetic
weights and on-disk format.

The reference runs vibert-capu.onnx through onnxruntime in mini-batches of <= 32 sentences
(core/gec_model.py:366-412): inputs input_ids / attention_mask / token_type_ids [B][L] and
input_offsets [B][W] (the first sub-token of every word), outputs logits [B][W][labels] and
detect_logits [B][W][detect classes].  The graph is the reference's own
convert_onnx/export_vibert_onnx.py Seq2LabelsModel: a BERT encoder (transformers BertModel,
FPTAI vibert-base-cased: 12 layers, hidden 768, 12 heads, intermediate 3072, GELU (erf),
LayerNorm eps 1e-12, vocabulary 38168 + 1 START token after special_tokens_fix), the
sequence output gathered at input_offsets, and two linear heads (classifier, detector).

Weights are SYNTHETIC (seeded numpy PCG64) under the Hugging Face state-dict names; no
checkpoint is available offline.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np


@dataclasses.dataclass
class VibertConfig:
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    vocab_size: int = 38169          # 38168 + START_TOKEN (special_tokens_fix)
    num_labels: int = 15
    num_detect_classes: int = 4
    layer_norm_eps: float = 1e-12

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self), indent=1)

    @staticmethod
    def from_json(text: str) -> "VibertConfig":
        return VibertConfig(**json.loads(text))

    def bert_config_json(self) -> dict:
        """transformers BertConfig fields of the encoder (the reference builds it with
        AutoConfig.from_pretrained(pretrained_name_or_path), export_vibert_onnx.py:100-104)."""
        return {"model_type": "bert", "architectures": ["BertModel"],
                "hidden_size": self.hidden_size, "num_hidden_layers": self.num_hidden_layers,
                "num_attention_heads": self.num_attention_heads,
                "intermediate_size": self.intermediate_size,
                "max_position_embeddings": self.max_position_embeddings,
                "type_vocab_size": self.type_vocab_size, "vocab_size": self.vocab_size - 1,
                "hidden_act": "gelu", "layer_norm_eps": self.layer_norm_eps,
                "hidden_dropout_prob": 0.1, "attention_probs_dropout_prob": 0.1,
                "pad_token_id": 0}


def vibert_base() -> VibertConfig:
    return VibertConfig()


def vibert_tiny() -> VibertConfig:
    """Small configuration of the same graph for fast tests."""
    return VibertConfig(hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                        intermediate_size=128, vocab_size=101)


def param_shapes(cfg: VibertConfig) -> "OrderedDict[str, Tuple[int, ...]]":
    s: "OrderedDict[str, Tuple[int, ...]]" = OrderedDict()
    H, I = cfg.hidden_size, cfg.intermediate_size
    e = "bert.embeddings."
    s[e + "word_embeddings.weight"] = (cfg.vocab_size, H)
    s[e + "position_embeddings.weight"] = (cfg.max_position_embeddings, H)
    s[e + "token_type_embeddings.weight"] = (cfg.type_vocab_size, H)
    s[e + "LayerNorm.weight"] = (H,)
    s[e + "LayerNorm.bias"] = (H,)
    for i in range(cfg.num_hidden_layers):
        p = f"bert.encoder.layer.{i}."
        for n in ("query", "key", "value"):
            s[p + f"attention.self.{n}.weight"] = (H, H)
            s[p + f"attention.self.{n}.bias"] = (H,)
        s[p + "attention.output.dense.weight"] = (H, H)
        s[p + "attention.output.dense.bias"] = (H,)
        s[p + "attention.output.LayerNorm.weight"] = (H,)
        s[p + "attention.output.LayerNorm.bias"] = (H,)
        s[p + "intermediate.dense.weight"] = (I, H)
        s[p + "intermediate.dense.bias"] = (I,)
        s[p + "output.dense.weight"] = (H, I)
        s[p + "output.dense.bias"] = (H,)
        s[p + "output.LayerNorm.weight"] = (H,)
        s[p + "output.LayerNorm.bias"] = (H,)
    s["bert.pooler.dense.weight"] = (H, H)
    s["bert.pooler.dense.bias"] = (H,)
    s["classifier.weight"] = (cfg.num_labels, H)
    s["classifier.bias"] = (cfg.num_labels,)
    s["detector.weight"] = (cfg.num_detect_classes, H)
    s["detector.bias"] = (cfg.num_detect_classes,)
    return s


def synth_weights(cfg: VibertConfig, seed: int = 20261018) -> Dict[str, np.ndarray]:
    """BERT-style init: N(0, 0.02) matrices / embeddings, zero-ish biases, LayerNorm near 1
    (heads scaled up so the label distribution is not flat)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = {}
    for name, shape in param_shapes(cfg).items():
        if "LayerNorm.weight" in name:
            w = rng.uniform(0.9, 1.1, size=shape)
        elif name.endswith(".bias"):
            w = rng.normal(0.0, 0.02, size=shape)
        elif name.startswith(("classifier", "detector")):
            w = rng.normal(0.0, 1.0 / math.sqrt(shape[1]), size=shape)
        else:
            w = rng.normal(0.0, 0.02 if "embeddings" in name else 1.0 / math.sqrt(shape[-1]),
                           size=shape)
        out[name] = np.ascontiguousarray(w, dtype=np.float32)
    return out


def save_model_dir(path: str, cfg: VibertConfig, weights: Dict[str, np.ndarray]) -> str:
    """vibert_config.json + vibert.safetensors (the engine's ViBERT format)."""
    from safetensors.numpy import save_file
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "vibert_config.json"), "w") as f:
        f.write(cfg.to_json())
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()},
              os.path.join(path, "vibert.safetensors"))
    return path


def vibert_flops(cfg: VibertConfig, B: int, L: int, W: int) -> float:
    H, I, nl = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    per_tok = 2.0 * (4 * H * H + 2 * H * I)
    att = 2.0 * 2 * L * L * H  # scores + context, all heads
    return nl * (B * L * per_tok + B * att) + 2.0 * B * W * H * (cfg.num_labels + cfg.num_detect_classes)
