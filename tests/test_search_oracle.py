"""Oracle search/hotword restatement vs the reference's own outputs (golden fixtures).

Fixtures were produced by tests/golden/make_golden.py running /root/reference's
`_ort_beam_search` (core/asr_engine.py:1023-1153), `_compute_token_entropy` (:1159-1181),
`decode_chunk` (:1209-1326) and `ContextGraph` (core/hotword_context.py:34-184).
"""
import glob
import json
import os

import numpy as np
import pytest

from oracle.search import HotwordGraph, beam_search, token_entropy
from synth_case import case_config, dec_joiner_weights, enc_out_for, np_decoder, np_joiner
from make_golden import checksum

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = sorted(glob.glob(os.path.join(GOLD, "search_*.json")))


def load_case(path):
    with open(path) as f:
        g = json.load(f)
    cfg = case_config(g["kind"])
    w = dec_joiner_weights(g["kind"], g["seed"])
    enc = enc_out_for(g["kind"], g["seed"], g["T"], cfg.joiner_dim)
    assert checksum(enc) == g["enc_checksum"], "synthetic input generator drifted"
    return g, cfg, w, enc


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_oracle_search_matches_reference(path):
    g, cfg, w, enc = load_case(path)
    graph = HotwordGraph(g["phrases"], g["scores"]) if g["hotwords"] else None
    toks, frames, lps, Tn, emit = beam_search(
        enc, lambda y: np_decoder(w, y), lambda e, d: np_joiner(w, e, d), g["beam"], graph)
    assert toks == g["token_ids"]
    assert frames == g["frames"]
    assert Tn == g["T_out"]
    np.testing.assert_allclose(lps, g["ys_log_probs"], rtol=0, atol=1e-9)
    ent = [token_entropy(e, cfg.vocab_size) for e in emit]
    assert ent == g["entropy"]


def test_oracle_hotword_walks_match_reference():
    with open(os.path.join(GOLD, "hotword_walks.json")) as f:
        g = json.load(f)
    graph = HotwordGraph(g["phrases"], g["scores"])
    for walk in g["walks"]:
        st = graph.root
        for tok, delta, node_score, is_root in walk["steps"]:
            d, st = graph.step(st, tok)
            assert d == delta
            assert st.node_score == node_score
            assert (st is graph.root) == is_root
        assert graph.finalize(st) == walk["finalize"]
