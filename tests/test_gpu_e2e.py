"""End-to-end parity of the real model shapes through the C ABI (libzasr.so) on an MI355X.

Zipformer-68M (BASELINE configs 2/3) and Zipformer-30M (configs 1/4), random-init weights,
seeded synthetic speech.  The oracle is fbank -> ZipformerOracle.encoder -> oracle
beam_search, i.e. the reference's `_ort_beam_search` (core/asr_engine.py:1023-1153, pinned by
tests/test_search_oracle.py) fed by the restated encoder (parity unpinned vs the absent ONNX
graph).

Tolerances (stated as the north star asks):
  fp32 mode      token ids and frames EXACT; token log-probs within 2e-3 absolute (the HIP
                 and torch fp32 encoders differ by ~1e-5 relative; log-softmax carries it);
                 per-token row statistics within 2e-3 relative; word texts and timestamps
                 exact, word probabilities / entropy fields within 2e-3
  search alone   HIP search on the ORACLE's encoder output vs the oracle search on the
                 same encoder output: tokens / frames exact, log-probs within 5e-4 (a token
                 log-prob is the difference of two f32 hypothesis scores of magnitude ~2000
                 after 800 frames, core/asr_engine.py:1099-1100,1121: f32 ulp 1.2e-4)
  bf16x6 mode    three-piece split-bf16 products (include/zasr.h ZASR_PRECISION_BF16X6):
                 token ids and frames EXACT vs the fp32 oracle on the three 68M chunks (greedy
                 and beam 8 + hotwords), like fp32
  bf16x3 mode    two-piece split (encoder_out ~3e-5 from the oracle vs ~4e-6 for fp32 /
                 bf16x6): statistical like bf16, bounded by 0.05 (measured 0.0 greedy, 0.01
                 beam 8 + hotwords; one near-tie of the 802-token chunk flips)
  bf16 modes     statistical: the token error rate (edit distance / reference tokens) vs the
                 fp32 oracle is measured, written to gpurun_out/bf16_token_error.json (kept
                 under profiles/) and bounded by 0.15 pooled over the chunks (measured
                 0.03-0.10; the bound catches a broken path, DESIGN.md §5 reports the rates)
"""
import json
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

HOTWORDS = os.path.join(os.path.dirname(__file__), "golden", "hotword_sample.txt")
M_SECS = (20.0, 33.0, 7.5)


@pytest.fixture(scope="module")
def need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def _speech(seconds, seed):
    from zasr.synth_audio import synth_speech
    return synth_speech(seconds, seed)


def edit_distance(a, b) -> int:
    """Levenshtein distance of two int sequences (numpy row DP)."""
    a = np.asarray(a, np.int64)
    b = np.asarray(b, np.int64)
    if a.size == 0 or b.size == 0:
        return int(max(a.size, b.size))
    prev = np.arange(b.size + 1, dtype=np.int64)
    j = np.arange(b.size + 1, dtype=np.int64)
    for i in range(1, a.size + 1):
        sub = prev[:-1] + (b != a[i - 1])
        cand = np.empty_like(prev)
        cand[0] = i
        cand[1:] = np.minimum(prev[1:] + 1, sub)
        prev = j + np.minimum.accumulate(cand - j)  # insertions: cummin of cand[k] + (j - k)
    return int(prev[-1])


def _first_divergence(a, b):
    for i, (x, y) in enumerate(zip(a, b)):
        if x != y:
            return i
    return min(len(a), len(b)) if len(a) != len(b) else -1


def _assert_same(r, ref, lp_tol, stat_tol, what):
    from oracle.search import raw_token_stats
    toks, frames, lps, T, emit = ref
    got = r.token_ids.tolist()
    assert r.T == T, (what, r.T, T)
    d = _first_divergence(got, toks)
    assert d < 0, (f"{what}: tokens diverge at {d} of {len(toks)} "
                   f"(frame {frames[d] if d < len(frames) else '-'}): "
                   f"got {got[max(0, d - 2):d + 3]} want {toks[max(0, d - 2):d + 3]}")
    assert r.frames.tolist() == frames, what
    np.testing.assert_allclose(r.log_probs, lps, atol=lp_tol, rtol=0, err_msg=what)
    for k, (st, e) in enumerate(zip(r.stats, emit)):
        want = np.array(raw_token_stats(e), np.float64)
        np.testing.assert_allclose(st, want, rtol=stat_tol, atol=1e-6, err_msg=f"{what} tok {k}")


def _hotword_phrases(V, emitted):
    """config 3's graph: the reference's hotword.txt (266 lines) tokenized by the syllable
    hash (bpe.model is absent) + n-grams the model emits (full matches happen)."""
    from oracle.search import parse_hotwords
    from synth_case import hotword_token_ids, ngram_phrases
    seqs, scores = hotword_token_ids(parse_hotwords(HOTWORDS), V)
    ng = ngram_phrases(emitted)
    return seqs + ng, scores + [2.0] * len(ng)


@pytest.fixture(scope="module")
def m_case(need_gpu):
    from model_fixtures import m_model
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from oracle.zipformer import ZipformerOracle
    cfg, w, path = m_model()
    orc = ZipformerOracle(cfg, w)
    chunks = [_speech(s, 1200 + i) for i, s in enumerate(M_SECS)]
    encs = [orc.encoder(fbank(c)) for c in chunks]
    greedy = [beam_search(e, orc.decoder, orc.joiner, 1) for e in encs]
    phrases, scores = _hotword_phrases(cfg.vocab_size, greedy[0][0])
    graph = HotwordGraph(phrases, scores)
    beam8 = [beam_search(e, orc.decoder, orc.joiner, 8, graph) for e in encs]
    return {"cfg": cfg, "w": w, "path": path, "orc": orc, "chunks": chunks, "encs": encs,
            "greedy": greedy, "beam8": beam8, "phrases": phrases, "scores": scores,
            "graph": graph}


def test_m_greedy_fp32_end_to_end(m_case):
    """68M greedy (config 2's method) in the fp32 parity mode: token-exact vs the oracle."""
    from zasr.binding import Recognizer
    rec = Recognizer(m_case["path"], "greedy_search", 1, precision="fp32")
    res = rec.decode(m_case["chunks"])
    for i, (r, ref) in enumerate(zip(res, m_case["greedy"])):
        _assert_same(r, ref, 2e-3, 2e-3, f"greedy chunk {i}")
    assert sum(len(g[0]) for g in m_case["greedy"]) > 100
    rec.close()


def test_m_beam8_hotwords_fp32_end_to_end(m_case):
    """68M modified beam search, beam 8, with the hotword.txt graph (config 3): token-exact
    vs the oracle, including hotword deltas, log-add merges and the final pick."""
    from zasr.binding import Recognizer
    rec = Recognizer(m_case["path"], "modified_beam_search", 8, hotwords=m_case["phrases"],
                     hotword_scores=m_case["scores"], precision="fp32")
    res = rec.decode(m_case["chunks"])
    for i, (r, ref) in enumerate(zip(res, m_case["beam8"])):
        _assert_same(r, ref, 2e-3, 2e-3, f"beam8+hw chunk {i}")
    rec.close()


@pytest.mark.parametrize("beam", [1, 8])
def test_m_search_on_oracle_encoder_out(m_case, beam):
    """The search alone at the real shape (V = 2000, D = 512, T' up to 823): HIP search on
    the oracle's encoder output == oracle search on it (tokens / frames exact)."""
    from oracle.search import beam_search
    from zasr.binding import Recognizer
    orc = m_case["orc"]
    kw = {"hotwords": m_case["phrases"], "hotword_scores": m_case["scores"]} if beam > 1 else {}
    rec = Recognizer(m_case["path"], "modified_beam_search", 8, precision="fp32", **kw)
    res = rec.search(m_case["encs"], beam=beam)
    for i, (r, e) in enumerate(zip(res, m_case["encs"])):
        ref = m_case["greedy"][i] if beam == 1 else m_case["beam8"][i]
        _assert_same(r, ref, 5e-4, 1e-3, f"search beam {beam} chunk {i}")
    rec.close()


def test_m_bf16_token_error_rate(m_case):
    """bf16 (config 2's benched precision) and bf16_enc (bf16 encoder, f32 joiner + search):
    token error rate vs the fp32 oracle, greedy and beam 8 + hotwords."""
    from zasr.binding import Recognizer
    ref = {"greedy": m_case["greedy"], "beam8_hotwords": m_case["beam8"]}
    report = {}
    for prec in ("bf16", "bf16_enc", "fp32", "bf16x3", "bf16x6", "f16x3"):
        for name, method, beam in (("greedy", "greedy_search", 1),
                                   ("beam8_hotwords", "modified_beam_search", 8)):
            kw = {"hotwords": m_case["phrases"], "hotword_scores": m_case["scores"]} if beam > 1 else {}
            rec = Recognizer(m_case["path"], method, beam, precision=prec, **kw)
            res = rec.decode(m_case["chunks"])
            rec.close()
            errs = [edit_distance(r.token_ids.tolist(), g[0]) for r, g in zip(res, ref[name])]
            n = [len(g[0]) for g in ref[name]]
            report[f"{prec}/{name}"] = {
                "token_error_rate": round(sum(errs) / max(1, sum(n)), 5),
                "per_chunk": [round(e / max(1, k), 5) for e, k in zip(errs, n)],
                "ref_tokens": n, "exact_chunks": sum(int(e == 0) for e in errs)}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/bf16_token_error.json", "w") as f:
        json.dump({"model": "zipformer-68m (random init)", "chunks_sec": M_SECS,
                   "reference": "fp32 oracle (fbank + torch encoder + reference search)",
                   "rates": report}, f, indent=1)
    for prec in ("fp32", "bf16x6", "f16x3"):
        assert report[f"{prec}/greedy"]["token_error_rate"] == 0.0, report
        assert report[f"{prec}/beam8_hotwords"]["token_error_rate"] == 0.0, report
    for name in ("greedy", "beam8_hotwords"):
        assert report[f"bf16x3/{name}"]["token_error_rate"] <= 0.05, report
    for k, v in report.items():
        assert v["token_error_rate"] <= 0.15, (k, v)


# ------------------------------------------------------------------ token-exact, widened
WIDE_CHUNKS = 18


@pytest.fixture(scope="module")
def m_wide(need_gpu):
    """The first 18 planner chunks of the benched hour (bench.make_chunks: 27-35 s each), the
    68M oracle's greedy and beam 8 + hotwords decodes of them (hotword.txt + n-grams the model
    emits, as m_case)."""
    import bench
    from model_fixtures import m_model
    from oracle.fbank import fbank
    from oracle.search import HotwordGraph, beam_search
    from oracle.zipformer import ZipformerOracle
    cfg, w, path = m_model(bench.WEIGHT_SEED)
    orc = ZipformerOracle(cfg, w)
    chunks = bench.make_chunks(WIDE_CHUNKS * 36.0 + 40.0, bench.AUDIO_SEED)[:WIDE_CHUNKS]
    encs = [orc.encoder(fbank(c)) for c in chunks]
    greedy = [beam_search(e, orc.decoder, orc.joiner, 1) for e in encs]
    phrases, scores = _hotword_phrases(cfg.vocab_size, greedy[0][0])
    graph = HotwordGraph(phrases, scores)
    beam8 = [beam_search(e, orc.decoder, orc.joiner, 8, graph) for e in encs]
    return {"path": path, "chunks": chunks, "greedy": greedy, "beam8": beam8,
            "phrases": phrases, "scores": scores, "orc": orc, "encs": encs, "graph": graph}


def _greedy_tie_margin(enc, orc, ref, got_toks, got_frames):
    """First frame where a greedy decode leaves the oracle's: the oracle's log-prob of its own
    choice minus that of the other decode's choice at that frame (both share the context up to
    it).  A rounding-level tie has a margin far below the logits' scale."""
    from oracle.search import BLANK, CTX
    toks, frames = ref[0], ref[1]
    a = dict(zip(frames, toks))
    b = dict(zip(got_frames, got_toks))
    ctx = [BLANK] * CTX
    for t in range(enc.shape[0]):
        x, y = a.get(t, BLANK), b.get(t, BLANK)
        if x != y:
            dec = orc.decoder(np.array([ctx[-CTX:]], dtype=np.int64))
            lg = orc.joiner(enc[t:t + 1], dec).astype(np.float64)[0]
            lp = lg - lg.max() - np.log(np.exp(lg - lg.max()).sum())
            return t, float(lp[x] - lp[y])
        if x != BLANK:
            ctx.append(x)
    return -1, 0.0


def _perturbed(enc, seed, rel=2.0 ** -20):
    """enc * (1 + rel * u), u in {-1, 0, 1} seeded: a relative change of ~1e-6, below the
    ~3e-6 by which two f32 encoders (the torch oracle, the GPU) differ on these chunks."""
    u = np.random.default_rng(seed).integers(-1, 2, size=enc.shape).astype(np.float64)
    return (enc.astype(np.float64) * (1.0 + rel * u)).astype(np.float32)


def _tie_audit(m_wide, fp32_recs, toks):
    """Every chunk where fp32 / f16x3 / bf16x6 leave the fp32 oracle, or f16x3 / bf16x6 leave
    the GPU fp32 mode, is checked to sit on an f32 rounding tie:
      greedy: the oracle's own log-prob margin at the first differing frame (< 1e-3);
      beam 8 + hotwords: the oracle itself changes its tokens when its encoder output is
        perturbed by ~1e-6 relative (_perturbed, two seeds) -- the chunk's search is chaotic at
        the f32 noise floor, so no f32 implementation can be held to one answer there -- or
        the oracle meets an EXACT tie at the beam boundary (the beam-th and next candidate
        scores equal in f32): the reference keeps whichever np.argpartition's introselect
        leaves in its last k slots, an order the HIP search (score desc, then flat index asc)
        does not reproduce.  Both show up here only in the n-gram hotword loops (phrases cut
        from the model's own emissions, e.g. 905 / 1709 repeated, matched every frame).
    For the GPU fp32 mode it also records whether its search on the oracle's encoder output
    gives the oracle's tokens, and the oracle's search on the GPU's encoder output the GPU's."""
    from oracle.search import beam_search
    orc, audit = m_wide["orc"], {}
    for name, beam, ref, graph in (("greedy", 1, m_wide["greedy"], None),
                                   ("beam8_hotwords", 8, m_wide["beam8"], m_wide["graph"])):
        for i, r in enumerate(ref):
            diff = {p: toks[(p, name)][i] != r[0] for p in ("fp32", "f16x3", "bf16x6")}
            diff_gpu = {p: toks[(p, name)][i] != toks[("fp32", name)][i] for p in ("f16x3", "bf16x6")}
            if not any(diff.values()) and not any(diff_gpu.values()):
                continue
            enc_o = m_wide["encs"][i]
            entry = {"differs_from_oracle": [p for p, d in diff.items() if d],
                     "differs_from_gpu_fp32": [p for p, d in diff_gpu.items() if d],
                     "edit_distance_fp32": edit_distance(toks[("fp32", name)][i], r[0])}
            if diff["fp32"]:
                rec = fp32_recs[name]
                enc_g = rec.encode_features([rec.fbank(m_wide["chunks"][i])])[0]
                n = min(len(enc_o), len(enc_g))
                entry["enc_max_rel_diff"] = float(np.max(np.abs(enc_g[:n] - enc_o[:n]) /
                                                         np.maximum(1.0, np.abs(enc_o[:n]))))
                entry["gpu_search_on_oracle_enc_exact"] = \
                    rec.search([enc_o], beam=beam)[0].token_ids.tolist() == r[0]
                entry["oracle_search_on_gpu_enc_equals_gpu"] = \
                    beam_search(enc_g, orc.decoder, orc.joiner, beam, graph)[0] == \
                    toks[("fp32", name)][i]
            if beam == 1:
                margins = {}
                for p in ("fp32", "f16x3", "bf16x6"):
                    if diff[p]:
                        t, m = _greedy_tie_margin(enc_o, orc, r, toks[(p, name)][i],
                                                  toks[(p, name, "frames")][i])
                        margins[p] = {"frame": t, "oracle_margin": m}
                entry["greedy_margins"] = margins
            else:
                flips = [beam_search(_perturbed(enc_o, sd), orc.decoder, orc.joiner, beam,
                                     graph)[0] != r[0] for sd in (1, 2)]
                entry["oracle_flips_under_1e-6_perturbation"] = flips
                ties = []
                beam_search(enc_o, orc.decoder, orc.joiner, beam, graph, ties=ties)
                entry["oracle_exact_boundary_tie_frames"] = ties
            audit[f"{name}/chunk{i}"] = entry
    return audit


@pytest.mark.timeout(900)
def test_m_token_exact_wide(m_wide):
    """token-exactness measured on >= 12 planner chunks (>= 1.5k greedy and
    >= 6k beam-8 tokens) vs the fp32 oracle, for fp32 and the token-exact modes (f16x3, bf16x6);
    bf16x3 / bf16 are reported.  Greedy must be exact chunk for chunk, or differ only at an
    oracle margin below 1e-3; beam 8 + hotwords may differ only on chunks whose oracle decode
    itself changes under a 1e-6 relative perturbation of its encoder output (_tie_audit).
    Writes gpurun_out/token_exact_wide.json (kept under profiles/)."""
    from zasr.binding import Recognizer
    ref = {"greedy": m_wide["greedy"], "beam8_hotwords": m_wide["beam8"]}
    n_tok = {k: sum(len(g[0]) for g in v) for k, v in ref.items()}
    assert n_tok["greedy"] >= 1500 and n_tok["beam8_hotwords"] >= 6000, n_tok
    report, toks = {}, {}
    fp32_recs = {}
    for prec in ("fp32", "f16x3", "bf16x6", "bf16x3", "bf16"):
        for name, method, beam in (("greedy", "greedy_search", 1),
                                   ("beam8_hotwords", "modified_beam_search", 8)):
            kw = {"hotwords": m_wide["phrases"], "hotword_scores": m_wide["scores"]} if beam > 1 else {}
            rec = Recognizer(m_wide["path"], method, beam, precision=prec, **kw)
            res = rec.decode(m_wide["chunks"])
            if prec == "fp32":
                fp32_recs[name] = rec
            else:
                rec.close()
            got = [r.token_ids.tolist() for r in res]
            toks[(prec, name)] = got
            toks[(prec, name, "frames")] = [r.frames.tolist() for r in res]
            errs = [edit_distance(g, r[0]) for g, r in zip(got, ref[name])]
            report[f"{prec}/{name}"] = {
                "token_error_rate": round(sum(errs) / max(1, n_tok[name]), 6),
                "exact_chunks": f"{sum(int(e == 0) for e in errs)}/{len(errs)}",
                "oracle_tokens": n_tok[name],
                "identical_to_gpu_fp32": None if prec == "fp32" else
                f"{sum(a == b for a, b in zip(got, toks[('fp32', name)]))}/{len(got)}"}
    audit = _tie_audit(m_wide, fp32_recs, toks)
    for r in fp32_recs.values():
        r.close()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/token_exact_wide.json", "w") as f:
        json.dump({"model": "zipformer-68m (random init, bench weights)",
                   "chunks": [round(len(c) / 16000.0, 2) for c in m_wide["chunks"]],
                   "reference": "fp32 oracle (numpy fbank + torch fp32 encoder + reference search)",
                   "rates": report, "tie_audit": audit}, f, indent=1)
    for k, e in audit.items():
        if k.startswith("greedy/"):
            for p, m in e["greedy_margins"].items():
                assert 0.0 <= m["oracle_margin"] < 1e-3, (k, p, e)
        else:
            assert any(e["oracle_flips_under_1e-6_perturbation"]) or \
                e["oracle_exact_boundary_tie_frames"], (k, e)
        if "enc_max_rel_diff" in e:
            assert e["enc_max_rel_diff"] <= 2e-3, (k, e)
    for prec in ("fp32", "f16x3", "bf16x6"):
        assert report[f"{prec}/greedy"]["token_error_rate"] <= 0.005, report
        assert report[f"{prec}/beam8_hotwords"]["token_error_rate"] <= 0.02, report


# ------------------------------------------------------------------ Zipformer-30M
@pytest.fixture(scope="module")
def s_case(need_gpu):
    from model_fixtures import s_model
    from oracle.zipformer import ZipformerOracle
    cfg, w, path = s_model()
    return {"cfg": cfg, "w": w, "path": path, "orc": ZipformerOracle(cfg, w)}


def test_s_encoder_matches_oracle(s_case):
    """30M encoder (ROVER model A, config 1's model): fp32 within 2e-3 * max(1, |ref|),
    bf16 within 0.05 * max(1, |ref|), ragged batch."""
    from oracle.fbank import fbank
    from zasr.binding import Recognizer
    feats = [fbank(_speech(s, 1300 + i)) for i, s in enumerate((17.0, 4.2, 29.0))]
    refs = [s_case["orc"].encoder(f) for f in feats]
    for prec, tol in (("fp32", 2e-3), ("bf16x6", 2e-3), ("f16x3", 2e-3), ("bf16x3", 2e-3),
                      ("bf16", 0.05)):
        rec = Recognizer(s_case["path"], "greedy_search", 1, precision=prec)
        got = rec.encode_features(feats)
        rec.close()
        for g, ref in zip(got, refs):
            assert g.shape == ref.shape
            err = float(np.max(np.abs(g - ref) / np.maximum(1.0, np.abs(ref))))
            assert err <= tol, (prec, err)


def test_s_plumbing_one_wav_through_dropin_decode_chunk(s_case, tmp_path):
    """Config 1: Zipformer-30M greedy on ONE 60 s 16 kHz WAV through the drop-in
    create_recognizer + decode_chunk (reference :903-1020, :1209-1326): the word dicts equal
    the oracle pipeline's (same BPE merge / timestamp / entropy code on oracle rows)."""
    import wave
    from oracle.fbank import fbank
    from oracle.search import beam_search
    from zasr.asr_engine import _words_from_search, create_recognizer, decode_chunk
    audio = _speech(60.0, 1401)
    wav = tmp_path / "one.wav"
    with wave.open(str(wav), "wb") as f:  # 16-bit PCM like a user's file
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes((np.clip(audio, -1, 1) * 32767).astype("<i2").tobytes())
    with wave.open(str(wav), "rb") as f:
        pcm = np.frombuffer(f.readframes(f.getnframes()), "<i2").astype(np.float32) / 32768.0
    rec = create_recognizer(s_case["path"], max_active_paths=1, precision="fp32")
    words = decode_chunk(rec, pcm, 12.0)
    orc = s_case["orc"]
    toks, frames, lps, T, emit = beam_search(orc.encoder(fbank(pcm)), orc.decoder, orc.joiner, 1)
    ref = _words_from_search(rec["id2token"], rec["vocab_size"], len(pcm), 12.0, toks, frames,
                             lps, T, emit)
    assert len(words) == len(ref) and len(ref) > 20
    for a, b in zip(words, ref):
        assert a["text"] == b["text"]
        for k in ("start", "end", "local_start", "local_end"):
            assert a[k] == pytest.approx(b[k], abs=1e-9), k
        for k in ("prob", "tsallis_max", "margin_min", "entropy_norm", "_conf"):
            assert a[k] == pytest.approx(b[k], abs=2e-3), k


def test_rover_30m_68m_matches_oracle(m_case, s_case):
    """Config 4 on the real shapes: 30M (model A) + 68M (model B), beam 8 each
    (core/asr_engine.py:2041-2047), one shared GPU fbank per chunk (:2346-2350), each model's
    words vs the oracle's, and the block vote vs rover_merge on the oracle words."""
    import copy
    from oracle.fbank import fbank
    from oracle.search import beam_search
    from zasr.asr_engine import _words_from_search, create_recognizer
    from zasr.rover import decode_chunks_rover, rover_merge
    ra = create_recognizer(s_case["path"], max_active_paths=8, precision="fp32")
    rb = create_recognizer(m_case["path"], max_active_paths=8, precision="fp32")
    chunks = [_speech(s, 1500 + i) for i, s in enumerate((21.0, 12.0))]
    offs = [0.0, 18.0]
    got = decode_chunks_rover(ra, rb, chunks, offs)
    for ci, (c, off) in enumerate(zip(chunks, offs)):
        f = fbank(c)
        per = []
        for rec, orc in ((ra, s_case["orc"]), (rb, m_case["orc"])):
            toks, frames, lps, T, emit = beam_search(orc.encoder(f), orc.decoder, orc.joiner, 8)
            per.append(_words_from_search(rec["id2token"], rec["vocab_size"], len(c), off,
                                          toks, frames, lps, T, emit))
        merged, dis = rover_merge(copy.deepcopy(per[0]), copy.deepcopy(per[1]))
        g_merged, g_dis = got[ci]
        assert [w["text"] for w in g_merged] == [w["text"] for w in merged], ci
        assert [round(w["start"], 9) for w in g_merged] == [round(w["start"], 9) for w in merged]
        assert g_dis == dis


def test_rover_device_passes_equal_host_route(m_case, s_case):
    """zasr.rover.rover_device_many (both models decode the HBM-resident chunks concurrently,
    each computing the fbank on the device, passes pipelined) == decode_chunks_rover (one
    shared GPU fbank per chunk through host memory) + merge_chunks_with_overlap, for every
    pass."""
    import torch
    from zasr.asr_engine import create_recognizer
    from zasr.merge import merge_chunks_with_overlap
    from zasr.rover import decode_chunks_rover, rover_device_many
    ra = create_recognizer(s_case["path"], max_active_paths=8, precision="bf16")
    rb = create_recognizer(m_case["path"], max_active_paths=8, precision="bf16")
    chunks = [_speech(s, 1600 + i) for i, s in enumerate((14.0, 9.5, 11.0))]
    lens = [c.shape[0] for c in chunks]
    d = torch.from_numpy(np.concatenate(chunks)).cuda()
    torch.cuda.synchronize()
    # the chunks' positions in HBM are their time offsets (packed back to back)
    poffs = np.cumsum([0] + lens[:-1]).tolist()
    got2 = decode_chunks_rover(ra, rb, chunks, [o / 16000.0 for o in poffs])
    ref2, _ = merge_chunks_with_overlap([{"words": m, "audio_start_abs": o / 16000.0,
                                          "audio_end_abs": (o + n) / 16000.0}
                                         for (m, _), o, n in zip(got2, poffs, lens)])
    passes = rover_device_many(ra["handle"], rb["handle"], ra, rb, d.data_ptr(), poffs, lens, 2, 8)
    passes += rover_device_many(ra["handle"], rb["handle"], ra, rb, d.data_ptr(), poffs, lens, 2,
                                8, sub_batches=2)
    passes += rover_device_many(ra["handle"], rb["handle"], ra, rb, d.data_ptr(), poffs, lens, 3,
                                8, passes_per_call=2)
    for words, dis, ta, tb in passes:
        assert [w["text"] for w in words] == [w["text"] for w in ref2]
        assert [w["start"] for w in words] == [w["start"] for w in ref2]
        assert dis == [len(x) for _, x in got2]
        assert ta > 0 and tb > 0
    assert len(ref2) > 0
