"""Seeded synthetic search cases shared by the golden-fixture generator and the tests.

A case = (joiner/decoder weights, encoder output, hotword phrases).  Decoder/joiner are
evaluated in plain numpy float32 here; the same functions back the "fake sessions" that
make_golden.py hands to the reference's `_ort_beam_search` (core/asr_engine.py:1023), which
only calls `.run(None, feeds)` on them (:1047, :1055, :1085, :1092).
"""
from __future__ import annotations

import math
import os
import sys
from typing import Dict, List, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(os.path.dirname(_HERE))
sys.path.insert(0, os.path.join(_REPO, "sherpa-vietnamese-asr_amd"))

from zasr.model import (ZipformerConfig, hash_tokenize_phrases, synth_weights,  # noqa: E402
                        zipformer_m, zipformer_tiny)

HOTWORD_FILE = os.path.join(_HERE, "hotword_sample.txt")


def case_config(kind: str) -> ZipformerConfig:
    return zipformer_tiny(64) if kind == "small" else zipformer_m()


# joiner blank-logit bias per case kind: "small"/"full" sit 1 nat below the model default
# (~25-40 % emission at beam 1, sparse at beam 8); "dense" (V = 2000, T' = 320) is tuned so
# that beam 8 emits ~150 tokens -- dedup, log-add merges and hotword matches at the real shape
def case_blank_bias(kind: str, V: int) -> float:
    return 2.2 if kind == "dense" else 0.5 * math.log(V)


def dec_joiner_weights(kind: str, seed: int) -> Dict[str, np.ndarray]:
    cfg = case_config(kind)
    w = synth_weights(cfg, seed, blank_bias=case_blank_bias(kind, cfg.vocab_size), dec_gain=1.0,
                      blank_row_gain=1.0)
    keep = ("decoder.", "decoder_proj.", "joiner.")
    return {k: v for k, v in w.items() if k.startswith(keep)}


def enc_out_for(kind: str, seed: int, T: int, D: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    base = rng.normal(0.0, 0.8, size=(T, D)).astype(np.float32)
    # slow drift so neighbouring frames correlate like real encoder output
    drift = np.cumsum(rng.normal(0.0, 0.15, size=(T, D)), axis=0).astype(np.float32)
    return (base + 0.3 * drift).astype(np.float32)


def np_decoder(w: Dict[str, np.ndarray], y: np.ndarray) -> np.ndarray:
    """Stateless decoder (context 2): embedding -> grouped conv(k=2, groups=D/4) -> relu -> proj."""
    y = np.asarray(y, dtype=np.int64)
    E = w["decoder.embedding.weight"]
    emb = E[np.clip(y, 0, None)] * (y >= 0)[..., None]  # (B, 2, D)
    B, C, D = emb.shape
    Wc = w["decoder.conv.weight"]  # (D, 4, 2)
    g = emb.reshape(B, C, D // 4, 4)  # input channels grouped by 4
    # out[b, o] = sum_{ci, tap} Wc[o, ci, tap] * emb[b, tap, 4*(o//4) + ci]
    gi = g[:, :, np.arange(D) // 4, :]  # (B, C, D, 4): for each out channel its group's inputs
    out = np.einsum("bcoi,oic->bo", gi, Wc).astype(np.float32)
    out = np.maximum(out, 0.0)
    return (out @ w["decoder_proj.weight"].T + w["decoder_proj.bias"]).astype(np.float32)


def np_joiner(w: Dict[str, np.ndarray], enc: np.ndarray, dec: np.ndarray) -> np.ndarray:
    x = np.tanh(enc + dec).astype(np.float32)
    return (x @ w["joiner.output_linear.weight"].T + w["joiner.output_linear.bias"]).astype(np.float32)


def hotword_token_ids(phrases: List[Tuple[str, float]], V: int):
    """Deterministic syllable -> id tokenization into [3, V) (real bpe.model is absent)."""
    return hash_tokenize_phrases(phrases, V)


def ngram_phrases(token_ids: List[int], every: int = 6, n_max: int = 3) -> List[List[int]]:
    """Phrases cut from a decoded token sequence (2..n_max consecutive tokens every `every`
    positions): hotwords the model actually emits, so full Aho-Corasick matches happen."""
    out = []
    for i in range(0, max(0, len(token_ids) - 1), every):
        n = 2 + (i // every) % (n_max - 1)
        ph = [int(t) for t in token_ids[i:i + n]]
        if len(ph) >= 2 and ph not in out:
            out.append(ph)
    return out


def boosted_phrases_from_case(enc_T: int, V: int, seed: int, n: int = 12):
    """Extra random phrases (token-id lists) so hotwords actually fire on random models."""
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    return [list(map(int, rng.integers(3, V, size=rng.integers(1, 4)))) for _ in range(n)]
