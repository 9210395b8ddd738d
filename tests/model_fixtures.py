"""Model directories for parity tests (synthetic weights, written to a temp dir)."""
from __future__ import annotations

import dataclasses
import math
import os
import tempfile

import numpy as np

from zasr.model import (WEIGHTS_VERSION, ZipformerConfig, save_model_dir, synth_tokens, synth_weights,
                        zipformer_m, zipformer_s, zipformer_tiny)

_CACHE = os.environ.get("ZASR_TEST_MODELS", os.path.join(tempfile.gettempdir(), "zasr_test_models"))


def model_dir(name: str, cfg: ZipformerConfig, weights) -> str:
    path = os.path.join(_CACHE, f"{name}_v{WEIGHTS_VERSION}")
    if not os.path.exists(os.path.join(path, "model.safetensors")):
        save_model_dir(path, cfg, weights, synth_tokens(cfg.vocab_size))
    return path


def tiny_model(seed: int = 3):
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, seed)
    return cfg, w, model_dir(f"tiny_{seed}", cfg, w)


def m_model(seed: int = 20261015):
    cfg = zipformer_m()
    w = synth_weights(cfg, seed)
    return cfg, w, model_dir(f"m_{seed}", cfg, w)


def search_case_model(kind: str, seed: int):
    """A model whose decoder/joiner are exactly the golden case's (tests/golden/synth_case.py);
    the encoder is a small stand-in (search-only tests never run it)."""
    from synth_case import case_config, dec_joiner_weights
    ccfg = case_config(kind)
    cfg = dataclasses.replace(zipformer_tiny(ccfg.vocab_size), name=f"search-{kind}",
                              decoder_dim=ccfg.decoder_dim, joiner_dim=ccfg.joiner_dim)
    w = synth_weights(cfg, 1)
    w.update(dec_joiner_weights(kind, seed))
    return cfg, model_dir(f"search_{kind}_{seed}", cfg, w)


def s_model(seed: int = 20261016):
    """Zipformer-30M (ROVER model A, zipformer-30m-rnnt-6000h shapes), random init."""
    cfg = zipformer_s()
    w = synth_weights(cfg, seed)
    return cfg, w, model_dir(f"s_{seed}", cfg, w)
