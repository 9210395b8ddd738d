"""The C word builder (csrc/words_ext.c, zasr._zasr_words) against the Python restatement
of decode_chunk's post-processing (zasr.asr_engine._words_from_search, itself pinned by the
reference's own word dicts in tests/test_host_logic.py): identical dicts -- values bit for
bit, keys in the same order -- on the reference-generated search goldens and on random
results with Vietnamese pieces, unknown ids, one-piece chunks and words longer than numpy's
128-element pairwise block."""
import glob
import json
import os

import numpy as np
import pytest

from zasr import asr_engine as ae
from zasr.model import synth_tokens

words_ext = pytest.importorskip("zasr._zasr_words")
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _stats_from_rows(rows):
    """(entropy, sum p^(1/3), top1, top2) of raw joiner rows, as the reference's
    _compute_token_entropy computes them (float32 numpy; the values are exact in f32)."""
    out = []
    for z in rows:
        z = np.asarray(z, np.float32)
        p = np.exp(z - np.max(z))
        p /= np.sum(p)
        srt = np.sort(p)[::-1]
        out.append([-float(np.sum(p * np.log(p + 1e-30))), float(np.sum(p ** (1.0 / 3.0))),
                    float(srt[0]), float(srt[1]) if len(srt) > 1 else 1e-10])
    return np.asarray(out, np.float32).reshape(-1, 4)


def _both(id2token, V, n, off, toks, frames, lps, T, stats):
    pieces, lowered = ae._token_tables(id2token)
    c = words_ext.words_from_search(pieces, lowered, V, n, off, np.asarray(toks, np.int32),
                                    np.asarray(frames, np.int32), np.asarray(lps, np.float64),
                                    T, np.asarray(stats, np.float32).reshape(-1, 4))
    py = ae._words_from_search(id2token, V, n, off, list(map(int, toks)), list(map(int, frames)),
                               list(map(float, lps)), T, ae.TokenStats.rows(stats))
    return c, py


def _same(c, py):
    assert len(c) == len(py)
    for a, b in zip(c, py):
        assert list(a) == list(b)  # key order
        for k in b:
            if isinstance(b[k], float):
                assert (a[k] == b[k]) or (a[k] != a[k] and b[k] != b[k]), (k, a[k], b[k])
                assert np.signbit(a[k]) == np.signbit(b[k]), k
            else:
                assert a[k] == b[k], k


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "search_*.json"))))
def test_goldens(path):
    from oracle.search import HotwordGraph, beam_search
    from synth_case import case_config, dec_joiner_weights, enc_out_for, np_decoder, np_joiner
    g = json.load(open(path))
    if "decode_chunk" not in g:
        pytest.skip("no decode_chunk words in this golden")
    cfg = case_config(g["kind"])
    w = dec_joiner_weights(g["kind"], g["seed"])
    enc = enc_out_for(g["kind"], g["seed"], g["T"], cfg.joiner_dim)
    graph = HotwordGraph(g["phrases"], g["scores"]) if g["hotwords"] else None
    toks, frames, lps, T, emit = beam_search(enc, lambda y: np_decoder(w, y),
                                             lambda e, d: np_joiner(w, e, d), g["beam"], graph)
    id2token = dict(enumerate(synth_tokens(cfg.vocab_size)))
    dc = g["decode_chunk"]
    c, py = _both(id2token, cfg.vocab_size, dc["n_samples"], dc["time_offset"], toks, frames,
                  lps, T, _stats_from_rows(emit))
    _same(c, py)
    ref = dc["words"]
    assert len(c) == len(ref)
    for a, b in zip(c, ref):
        assert set(a) == set(b)


VI = ["▁Xin", "▁chào", "▁ĐƯỜNG", "ng", "▁Việt", "ời", "▁", " ", " Hà", "Nội", "▁ỦY", "BAN",
      "▁<unk>", "ữ", "▁Ơ", "Ố"]


@pytest.mark.parametrize("seed", range(12))
def test_random_results(seed):
    rng = np.random.default_rng(seed)
    V = int(rng.integers(20, 300))
    id2token = {i: (VI[i % len(VI)] + (str(i) if i % 5 else "")) for i in range(V) if i % 17 != 3}
    n = int(rng.integers(1, 600))
    if seed == 0:
        n = 1
    if seed == 1:  # one word of 300 pieces (numpy's pairwise split past 128)
        id2token = {i: f"x{i}" for i in range(V)}
        id2token[0] = "▁start"
    toks = rng.integers(0, V + 5, n)  # ids past the table and missing ids -> ""
    if seed == 1:
        toks[0] = 0
    T = int(rng.integers(n, 4 * n + 2))
    frames = np.sort(rng.choice(T, n, replace=False)) if n <= T else np.arange(n)
    lps = -np.abs(rng.standard_normal(n)) * 3
    stats = np.stack([rng.random(n) * 5, rng.random(n) * 40, rng.random(n),
                      rng.random(n) * 0.3], 1).astype(np.float32)
    n_samples = int(rng.integers(16000, 560000))
    off = float(rng.random() * 3000)
    c, py = _both(id2token, V, n_samples, off, toks, frames, lps, T, stats)
    assert len(py) >= 1
    _same(c, py)


def test_empty_and_no_frames():
    id2token = {0: "▁a", 1: "b"}
    for toks, T in (([], 10), ([0, 1], 0)):
        c, py = _both(id2token, 2, 16000, 0.0, toks, list(range(len(toks))), [-0.1] * len(toks),
                      T, np.zeros((len(toks), 4), np.float32))
        assert c == py == []


def test_round4_equals_python_round():
    """The builder's round(x, 4) (an exact FMA split of x * 10^4, no string round trip)
    against Python's round on random values over 24 decades, values one ulp either side of
    every 4-decimal midpoint in [-20, 20], signed zeros and the large-value route."""
    rng = np.random.default_rng(0)
    mids = np.arange(-200000, 200000) / 10000.0 + 0.00005
    xs = np.concatenate([rng.random(100000), rng.random(50000) * 100 - 50,
                         10 ** rng.uniform(-12, 11, 50000) * rng.choice([-1, 1], 50000), mids,
                         np.nextafter(mids, np.inf), np.nextafter(mids, -np.inf),
                         [0.0, -0.0, 1e-300, -1e-300, 5e-5, -5e-5, 0.99995, 4.5e11, -7e12, 1e20]])
    for x in xs.tolist():
        a, b = words_ext.round4(x), round(x, 4)
        assert a == b and np.signbit(a) == np.signbit(b), (x, a, b)


def test_table_checks():
    """mismatched table lengths raise ValueError, non-str entries TypeError (the
    Python path's behaviour), instead of reading past the lowered list or crashing."""
    tok = np.array([1, 2], np.int32)
    fr = np.array([0, 3], np.int32)
    lp = np.zeros(2, np.float64)
    st = np.zeros((2, 4), np.float32)
    with pytest.raises(ValueError):
        words_ext.words_from_search(["a", "b", "c"], ["a", "b"], 3, 16000, 0.0, tok, fr, lp, 10, st)
    with pytest.raises(TypeError):
        words_ext.words_from_search(["a", 5, "c"], ["a", "b", "c"], 3, 16000, 0.0, tok, fr, lp, 10, st)
