"""Generate golden search fixtures by running the REFERENCE's own Python.

Run in the build container only (needs /root/reference; the GPU box never runs this):

    python tests/golden/make_golden.py

It imports `core.asr_engine` and `core.hotword_context` from /root/reference and drives
`_ort_beam_search` (core/asr_engine.py:1023-1153) and `decode_chunk` (:1209-1326) with
duck-typed numpy "sessions" (only `.run(None, feeds)` is used: :1047, :1055, :1085, :1092)
over seeded synthetic decoder/joiner weights and encoder outputs (tests/golden/synth_case.py).
Hotword graphs are the reference's own `ContextGraph` (core/hotword_context.py:34-184) built
from `hotword.txt` phrases (tokenized by a deterministic syllable hash: bpe.model is absent)
plus random token phrases.

Outputs: tests/golden/search_*.json, tests/golden/hotword_walks.json.  Each fixture stores
the case seeds, a checksum of the regenerated inputs, and the reference outputs.
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import sys
import contextlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from synth_case import (HOTWORD_FILE, boosted_phrases_from_case, case_config,  # noqa: E402
                        dec_joiner_weights, enc_out_for, hotword_token_ids, ngram_phrases,
                        np_decoder, np_joiner)

REF = "/root/reference"


def _import_reference():
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import core.asr_engine as ae  # noqa: F401
        import core.hotword_context as hc  # noqa: F401
    return ae, hc


class _Sess:
    def __init__(self, fn):
        self.fn = fn

    def run(self, _outs, feeds):
        return self.fn(feeds)


def checksum(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def case_inputs(kind, seed, T):
    cfg = case_config(kind)
    w = dec_joiner_weights(kind, seed)
    enc = enc_out_for(kind, seed, T, cfg.joiner_dim)
    return cfg, w, enc


def phrases_for(hc, kind, seed, V, with_hw, emitted=None):
    if not with_hw:
        return [], []
    seqs, scores = hotword_token_ids(hc.parse_hotwords_file(HOTWORD_FILE, 1.5), V)
    extra = boosted_phrases_from_case(0, V, seed)
    seqs = seqs + extra
    scores = scores + [2.0 + 0.25 * (i % 3) for i in range(len(extra))]
    if emitted:  # n-grams the model emits without hotwords: full matches at V = 2000
        ng = ngram_phrases(emitted)
        seqs = seqs + ng
        scores = scores + [1.5 + 0.5 * (i % 2) for i in range(len(ng))]
    return seqs, scores


def full_matches(hc, seqs, scores, toks):
    """Completed phrases along the decoded tokens (the reference's non-strict walk: a full
    match returns the root with a positive delta)."""
    if not seqs:
        return 0
    g = hc.ContextGraph()
    g.build(seqs, scores)
    st, n = g.root, 0
    for t in toks:
        if t == 2:
            continue
        d, st = g.forward_one_step(st, t)
        n += int(st is g.root and d > 0)
    return n


def run_case(ae, hc, kind, seed, T, beam, with_hw, dump_chunk=False, emitted=None):
    cfg, w, enc = case_inputs(kind, seed, T)
    V = cfg.vocab_size
    seqs, scores = phrases_for(hc, kind, seed, V, with_hw, emitted)
    graph = None
    if seqs:
        graph = hc.ContextGraph()
        graph.build(seqs, scores)
    rec = {
        "enc_sess": _Sess(lambda f: [enc[None], np.array([enc.shape[0]], dtype=np.int64)]),
        "dec_sess": _Sess(lambda f: [np_decoder(w, f["y"])]),
        "joi_sess": _Sess(lambda f: [np_joiner(w, f["encoder_out"], f["decoder_out"])]),
        "vocab_size": V, "dec_cache": {}, "context_graph": graph,
        "id2token": {i: t for i, t in enumerate(_tokens(V))}, "max_active_paths": beam,
    }
    feats = np.zeros((4 * T + 8, 80), dtype=np.float32)
    toks, frames, lps, Tn, emit = ae._ort_beam_search(rec, feats, beam)
    ent = [ae._compute_token_entropy(e, V) for e in emit]
    out = {
        "kind": kind, "seed": seed, "T": T, "beam": beam, "hotwords": bool(seqs),
        "enc_checksum": checksum(enc), "V": V,
        "phrases": seqs, "scores": scores,
        "token_ids": [int(t) for t in toks], "frames": [int(f) for f in frames],
        "ys_log_probs": [float(x) for x in lps], "T_out": int(Tn),
        "entropy": ent,
        "hotword_full_matches": full_matches(hc, seqs, scores, toks),
    }
    if dump_chunk:
        rec["dec_cache"] = {}
        n_samples = 160 * (4 * T + 8) - 80
        words = ae.decode_chunk(rec, np.zeros(n_samples, dtype=np.float32), 12.5,
                                precomputed_features=feats)
        out["decode_chunk"] = {"n_samples": n_samples, "time_offset": 12.5,
                               "words": _jsonable(words)}
    return out


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, (np.integer,)):
        return int(x)
    return x


def _tokens(V):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "sherpa-vietnamese-asr_amd"))
    from zasr.model import synth_tokens
    return synth_tokens(V)


def hotword_walks(hc, V=64, seed=5):
    seqs, scores = hotword_token_ids(hc.parse_hotwords_file(HOTWORD_FILE, 1.5), V)
    extra = boosted_phrases_from_case(0, V, seed, n=20)
    seqs, scores = seqs + extra, scores + [1.0 + 0.5 * (i % 4) for i in range(len(extra))]
    g = hc.ContextGraph()
    g.build(seqs, scores)
    rng = np.random.Generator(np.random.PCG64(seed))
    phrase_toks = sorted({t for s in seqs for t in s})
    walks = []
    for _ in range(40):
        st = g.root
        steps = []
        for _ in range(30):
            t = int(rng.choice(phrase_toks)) if rng.random() < 0.8 else int(rng.integers(3, V))
            d, st = g.forward_one_step(st, t)
            steps.append([t, float(d), float(st.node_score), st is g.root])
        walks.append({"steps": steps, "finalize": float(g.finalize(st))})
    return {"V": V, "phrases": seqs, "scores": scores, "walks": walks}


def dense_cases(ae, hc, outdir):
    """V = 2000, T' = 320, blank bias tuned for ~150 beam-8 emissions; the hotword graph is
    hotword.txt + random phrases + n-grams of the no-hotword output (full matches)."""
    for beam in (4, 8):
        seed = 3001 + beam
        base = run_case(ae, hc, "dense", seed, 320, beam, False, dump_chunk=True)
        hw = run_case(ae, hc, "dense", seed, 320, beam, True, dump_chunk=True,
                      emitted=base["token_ids"])
        for res, tag in ((base, "nohw"), (hw, "hw")):
            name = f"search_dense_b{beam}_{tag}.json"
            with open(os.path.join(outdir, name), "w") as f:
                json.dump(res, f)
            print(name, "tokens:", len(res["token_ids"]), "T':", res["T_out"],
                  "full hotword matches:", res["hotword_full_matches"])


def main():
    ae, hc = _import_reference()
    outdir = HERE
    if "--dense-only" in sys.argv:
        dense_cases(ae, hc, outdir)
        return
    dense_cases(ae, hc, outdir)
    cases = []
    for kind, T in (("small", 60), ("full", 100)):
        for beam in (1, 4, 8):
            for hw in (False, True):
                seed = 101 + beam + (50 if hw else 0) + (1000 if kind == "full" else 0)
                cases.append((kind, seed, T, beam, hw))
    for kind, seed, T, beam, hw in cases:
        res = run_case(ae, hc, kind, seed, T, beam, hw, dump_chunk=(beam in (1, 8)))
        name = f"search_{kind}_b{beam}_{'hw' if hw else 'nohw'}.json"
        with open(os.path.join(outdir, name), "w") as f:
            json.dump(res, f)
        print(name, "tokens:", len(res["token_ids"]), "T':", res["T_out"])
    with open(os.path.join(outdir, "hotword_walks.json"), "w") as f:
        json.dump(hotword_walks(hc), f)
    print("hotword_walks.json")


if __name__ == "__main__":
    main()
