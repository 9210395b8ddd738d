"""Paths that real weights or real inputs select, each run on the GPU.

* Checked launches: every kernel launch is followed by the runtime's launch status
  (common.h ZASR_LAUNCH); a refused configuration surfaces as ZasrError, not as a decode that
  reads a workspace the kernel never wrote.
* f16x3 weight-range routing: the one-accumulator f16x3 kernels (fused FFN, row-resident
  GEMM, fused ConvNeXt MLP) scale the weight's fp16 hi piece by 2^11, exact for |w| < 32; a
  layer with |w| >= 31 keeps the two-accumulator GEMMs.  Random 1/sqrt(fan_in) weights never
  get there, trained ones can: here one FFN, the projections of one layer and the ConvNeXt
  pw1 carry a 40, and the encoder must still match the oracle (2e-3 * max(1, |ref|)) and
  decode the tokens the fp32 mode decodes.
* No decoder-context table: a vocabulary whose V^2 x D table exceeds ZASR_DEC_TABLE_MAX_GB
  runs the per-frame decoder (decjoin_kernel) + joiner + search step; forced here with the
  limit at 0, against the goldens made by the reference's own _ort_beam_search.
* The HIP fbank pinned to the reference's own outputs: the browser worker's computeFbank
  (offline_pwa/static/js/pure-ort-asr-worker.js:470-519, tests/golden/fbank_js.npz) uses
  Hz-linear triangles (:369-397) where knf uses mel-linear ones; with those triangles loaded
  (zasr_fbank_set_mel_banks) the kernel's log-mel output is held to the worker's outputs.
"""
import json
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def need_gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def _speech(seconds, seed):
    from zasr.synth_audio import synth_speech
    return synth_speech(seconds, seed)


# ------------------------------------------------------------------ checked launches
def test_checked_launch_reports_refused_config(need_gpu):
    from zasr.binding import ZasrError, selftest_launch
    selftest_launch(64)
    selftest_launch(1024)
    with pytest.raises(ZasrError, match="launch failed"):
        selftest_launch(2048)  # over the 1024-thread block limit: the runtime refuses it
    selftest_launch(256)  # the refusal is not sticky: the next launch runs


# ------------------------------------------------------------------ f16x3 weight ranges
HOT = 40.0  # >= 31: outside the one-accumulator kernels' exact range

HOT_TENSORS = [
    # a fused-FFN layer (stack 2, d = 384) -> the GEMM pair
    ("encoder.encoders.2.encoder.layers.0.feed_forward1.in_proj.weight", (3, 5)),
    # projections the row-resident GEMM takes at K = 384 -> the tiled gemm_x3
    ("encoder.encoders.2.encoder.layers.0.self_attn_weights.in_proj.weight", (7, 11)),
    ("encoder.encoders.2.encoder.layers.0.conv_module1.out_proj.weight", (2, 9)),
    ("encoder.encoders.2.encoder.layers.0.nonlin_attention.in_proj.weight", (300, 17)),
    # the ConvNeXt MLP -> convnext_mlp_h3_kernel (two accumulators)
    ("encoder_embed.convnext.pointwise_conv1.weight", (10, 20, 0, 0)),
]


@pytest.fixture(scope="module")
def hot_m(need_gpu, tmp_path_factory):
    from model_fixtures import m_model
    from zasr.model import save_model_dir, synth_tokens
    cfg, w, path = m_model()
    hot = dict(w)
    for name, idx in HOT_TENSORS:
        t = np.array(hot[name], dtype=np.float32, copy=True)
        t[idx] = HOT
        hot[name] = t
    d = str(tmp_path_factory.mktemp("hot_m"))
    save_model_dir(d, cfg, hot, synth_tokens(cfg.vocab_size))
    return cfg, w, path, hot, d


def test_f16x3_weight_range_routes(hot_m):
    from zasr.binding import Recognizer
    cfg, w, path, hot, d = hot_m
    base = Recognizer(path, "greedy_search", 1, precision="f16x3")
    rb = base.routes()
    base.close()
    rec = Recognizer(d, "greedy_search", 1, precision="f16x3")
    rh = rec.routes()
    rec.close()
    # the seeded weights take every one-accumulator kernel they fit
    assert rb["ffn_gemm_pair"] == 0 and rb["gemm_x3_range"] == 0 and rb["cnx_ffn_h3"] == 1
    assert rb["ffn_fused_h3"] == 48 and rb["gemm_h3r"] > 0 and rb["dec_table"] == 1
    # one FFN, the layer's K = 384 projections and the ConvNeXt MLP leave them
    assert rh["ffn_gemm_pair"] == 1 and rh["ffn_fused_h3"] == rb["ffn_fused_h3"] - 1
    assert rh["gemm_x3_range"] == 3
    assert rh["gemm_h3r"] == rb["gemm_h3r"] - rh["gemm_x3_range"]
    assert rh["cnx_ffn_h3"] == 0


def test_f16x3_weight_range_encoder_matches_oracle(hot_m):
    from oracle.fbank import fbank
    from oracle.zipformer import ZipformerOracle
    from zasr.binding import Recognizer
    cfg, w, path, hot, d = hot_m
    rec = Recognizer(d, "greedy_search", 1, precision="f16x3")
    feats = [fbank(_speech(12.3, 5)), fbank(_speech(3.1, 6))]
    got = rec.encode_features(feats)
    rec.close()
    orc = ZipformerOracle(cfg, hot)
    for f, g in zip(feats, got):
        ref = orc.encoder(f)
        assert g.shape == ref.shape
        err = np.max(np.abs(g - ref) / np.maximum(1.0, np.abs(ref)))
        assert err <= 2e-3, f"encoder max scaled error {err}"


@pytest.mark.parametrize("method,beam", [("greedy_search", 1), ("modified_beam_search", 4)])
def test_f16x3_weight_range_tokens_equal_fp32(hot_m, method, beam):
    from zasr.binding import Recognizer
    cfg, w, path, hot, d = hot_m
    chunks = [_speech(21.0, 41), _speech(7.5, 42), _speech(2.2, 43)]
    want = Recognizer(d, method, beam, precision="fp32").decode(chunks)
    rec = Recognizer(d, method, beam, precision="f16x3")
    got = rec.decode(chunks)
    assert rec._fallback is None  # decoded in f16x3, not re-run in bf16x6
    rec.close()
    assert sum(r.token_ids.size for r in want) > 20
    for a, b in zip(got, want):
        assert a.token_ids.tolist() == b.token_ids.tolist()
        assert a.frames.tolist() == b.frames.tolist()
        np.testing.assert_allclose(a.log_probs, b.log_probs, atol=5e-4, rtol=0)


# ------------------------------------------------------------------ no decoder table
CASES = sorted(f for f in os.listdir(GOLD) if f.startswith("search_") and f.endswith(".json"))


@pytest.mark.parametrize("name", CASES)
def test_search_without_decoder_table_matches_reference_golden(need_gpu, monkeypatch, name):
    """ZASR_DEC_TABLE_MAX_GB=0: no V^2 x D table, every frame runs decjoin_kernel (Embedding
    -> grouped Conv1d -> ReLU -> decoder_proj for every live slot, then tanh(enc + dec) as J),
    the path a vocabulary too large for the table takes; same goldens as the table path."""
    from model_fixtures import search_case_model
    from synth_case import case_config, enc_out_for
    from zasr.binding import Recognizer
    with open(os.path.join(GOLD, name)) as f:
        g = json.load(f)
    cfg, mdir = search_case_model(g["kind"], g["seed"])
    enc = enc_out_for(g["kind"], g["seed"], g["T"], case_config(g["kind"]).joiner_dim)
    monkeypatch.setenv("ZASR_DEC_TABLE_MAX_GB", "0")
    for prec in ("fp32", "f16x3"):
        rec = Recognizer(mdir, "modified_beam_search", 8,
                         hotwords=g["phrases"] if g["hotwords"] else None,
                         hotword_scores=g["scores"] if g["hotwords"] else None, precision=prec)
        assert rec.routes()["dec_table"] == 0
        r = rec.search([enc], beam=g["beam"])[0]
        rec.close()
        assert r.T == g["T_out"]
        assert r.token_ids.tolist() == g["token_ids"], prec
        assert r.frames.tolist() == g["frames"], prec
        np.testing.assert_allclose(r.log_probs, g["ys_log_probs"], atol=5e-4, rtol=0)


# ------------------------------------------------------------------ fbank vs the JS run
def test_fbank_kernel_matches_reference_js_run(need_gpu):
    """fbank_kernel with the worker's Hz triangles vs the worker's own outputs on the nine
    fixture inputs (lengths 1 .. 480000, silence, a tone).  Bounds: 5e-5 in log energy where
    the reference is above -10 (its f32 arithmetic: ~50 f32 ulps of the energy), 5e-4 overall
    (quiet frames near the 2^-23 floor, where the DC removal and the power cancel in f32) --
    the bounds the CPU restatement meets in tests/test_fbank_oracle.py."""
    from make_golden_fbank_js import fbank_js_inputs
    from model_fixtures import tiny_model
    from oracle.fbank import mel_banks_js
    from zasr.binding import Recognizer
    cfg, w, path = tiny_model()
    rec = Recognizer(path, "greedy_search", 1)
    z = np.load(os.path.join(GOLD, "fbank_js.npz"))
    knf = {name: rec.fbank(x) for name, x in fbank_js_inputs()}
    rec.set_mel_banks(mel_banks_js())
    worst = {}
    for name, x in fbank_js_inputs():
        ref = z[name]
        got = rec.fbank(x)
        assert got.shape == ref.shape, name
        if not ref.size:
            continue
        d = np.abs(got - ref)
        worst[name] = float(d.max())
        assert d.max() <= 5e-4, (name, float(d.max()))
        assert d[ref > -10.0].max(initial=0.0) <= 5e-5, name
    assert len(worst) >= 7
    # the override is what moved the kernel onto the worker's outputs (the default mel
    # triangles differ from them by up to ~1e-2 on speech)
    assert max(float(np.abs(knf[n] - z[n]).max()) for n in worst if n != "zeros_1600") > 1e-3
    rec.close()
