"""The stage engines opened from reference-layout ONNX directories on the MI355X
(tests/golden/write_stage_onnx.py layouts; the reader itself is pinned bit-exactly on CPU in
tests/test_stage_onnx.py):

* Silero VAD: VadSession on a dir holding only silero_vad_16k_op15.onnx (the If-branch
  layout) gives the same probabilities, bit for bit, as on the safetensors dir of the same
  weights; zasr.dropin.install(engine, vad_module=...) with the module's BASE_DIR pointing at
  a reference-layout tree (models/silero-vad/silero_vad_16k_op15.onnx) serves
  get_vad_segments from it with the safetensors route's segments.
* ViBERT: vibert-capu.onnx -> logits / detect logits bit-identical to the safetensors dir.
* CAM++: campplus_cn_en_common_200k.onnx with the exporter's Conv+BN fusion -> embeddings
  within the reference's rel_l2 2e-4 of the f64 oracle on the unfused weights (the fused
  weights are rounded differently, so not bitwise)."""
import os
import sys
import types

import numpy as np
import pytest

from conftest import gpu_available

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    if not gpu_available():
        pytest.skip("no GPU")


def test_silero_onnx_dir_equals_safetensors_and_install_route(gpu, tmp_path, monkeypatch):
    from write_stage_onnx import write_silero
    import zasr.vad_utils as vu
    from zasr.binding import VadSession
    from zasr.dropin import install
    from zasr.silero import SileroConfig, save_model_dir, synth_weights
    from zasr.synth_audio import synth_speech
    cfg = SileroConfig()
    w = synth_weights(cfg, 41)
    st_dir = save_model_dir(str(tmp_path / "st"), cfg, w)
    base = tmp_path / "ref"
    write_silero(str(base / "models" / "silero-vad"), w, "if")
    audios = [synth_speech(37.0, 5), synth_speech(12.5, 6)]
    a, b = VadSession(st_dir), VadSession(str(base / "models" / "silero-vad"))
    try:
        pa, pb = a.probs(audios, auto_boost=True), b.probs(audios, auto_boost=True)
    finally:
        a.close()
        b.close()
    for x, y in zip(pa, pb):
        assert np.array_equal(x, y)
    monkeypatch.setenv("ZASR_VAD_MODEL_DIR", st_dir)
    vu.unload_vad_model()
    want = [vu.get_vad_segments(x) for x in audios]
    monkeypatch.delenv("ZASR_VAD_MODEL_DIR")
    vu.unload_vad_model()
    ref_vad = types.ModuleType("core.vad_utils")
    ref_vad.BASE_DIR = str(base)
    ref_engine = types.ModuleType("core.asr_engine")
    try:
        install(ref_engine, vad_module=ref_vad)
        got = [ref_vad.get_vad_segments(x) for x in audios]
    finally:
        vu.unload_vad_model()
        vu.set_base_dir(None)
    assert got == want
    assert all(len(s) >= 1 for s in got)


def test_vibert_onnx_dir_equals_safetensors(gpu, tmp_path):
    from write_stage_onnx import write_vibert
    from zasr.binding import VibertSession
    from zasr.pipeline import vibert_feeds
    from zasr.vibert import save_model_dir, synth_weights, vibert_tiny
    import json
    cfg = vibert_tiny()
    w = synth_weights(cfg, 42)
    st = VibertSession(save_model_dir(str(tmp_path / "st"), cfg, w))
    write_vibert(str(tmp_path / "ox"), w)
    with open(tmp_path / "ox" / "config.json", "w") as f:
        json.dump({"num_attention_heads": cfg.num_attention_heads}, f)
    ox = VibertSession(str(tmp_path / "ox"))
    try:
        rng = np.random.default_rng(3)
        batch = [[f"w{int(x)}" for x in rng.integers(0, 300, int(n))] for n in rng.integers(3, 60, 40)]
        feeds = vibert_feeds(batch, cfg.vocab_size)
        la, da = st.run(None, feeds)
        lb, db = ox.run(None, feeds)
    finally:
        st.close()
        ox.close()
    assert np.array_equal(la, lb) and np.array_equal(da, db)


def test_campp_fused_onnx_dir_matches_oracle(gpu, tmp_path):
    import torch
    from oracle.campplus import CamppOracle
    from write_stage_onnx import write_campp
    from zasr.binding import CamppEmbedder
    from zasr.campp import CamppConfig, synth_weights
    cfg = CamppConfig()
    w = synth_weights(cfg, 43)
    write_campp(str(tmp_path / "ox"), w, fused=True)
    emb = CamppEmbedder(str(tmp_path / "ox"))
    try:
        x = np.random.default_rng(4).normal(size=(6, 150, 80)).astype(np.float32)
        got = emb.embed(x)
    finally:
        emb.close()
    torch.set_num_threads(8)
    exact = CamppOracle(cfg, w, dtype=np.float64).embed(x)
    # the reference's CAM++ acceptance number (core/calibration.py:71-78: rel_l2 <= 2e-4)
    # against the exact embedding of the unfused weights
    rel = float(np.linalg.norm(got - exact) / np.linalg.norm(exact))
    assert rel <= 2e-4, rel
