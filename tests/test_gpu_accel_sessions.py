"""CAM++ and ViBERT reached through the reference's own session factory.

zasr.dropin.install(engine, accel_module=...) wraps `create_ort_session`
(core/hardware_accel.py:555): the diarizer's "CAM++ speaker embedding" session
(core/speaker_diarization_senko_campp_optimized.py:364-368) and GecBERTModel's "ViBERT
punctuation" session (core/gec_model.py:168-172) come back as libzasr.so engines.  Here the
returned sessions are driven with the callers' own call shapes -- the diarizer's warm-up
run(['embs'], {'feats': zeros[1, 150, 80]}) (:381) and batched run(['embs'], {'feats':
[N, T, 80]}) (:604); GecBERTModel's run(None, feeds) (core/gec_model.py:387, :397) -- on
reference-layout model files (tests/golden/write_stage_onnx.py; the real files are absent), and
compared with the fixtures made by the reference's own CAMPPlus / Seq2LabelsModel classes
(campp_golden.npz, vibert_golden.npz) at the reference's GPU acceptance tolerances
(core/calibration.py:71-78, :95-101).  The stage any other caller names (pyannote, DNSMOS)
reaches the reference's own function.
"""
import json
import os
import types

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
CAMPP = np.load(os.path.join(GOLDEN, "campp_golden.npz"))
VIBERT = np.load(os.path.join(GOLDEN, "vibert_golden.npz"))
REF_GPU = {"CUDAExecutionProvider", "OpenVINOExecutionProvider", "DmlExecutionProvider",
           "ROCMExecutionProvider"}  # core/hardware_accel.py:468-469


@pytest.fixture(scope="module")
def accel():
    if not gpu_available():
        pytest.skip("no GPU")
    from zasr.dropin import install
    passed = []
    mod = types.ModuleType("core.hardware_accel")

    def create_ort_session(ort_module, model_path, sess_options, policy="cpu", stage=""):
        passed.append((model_path, stage))
        return "reference-session", {"actual_provider": "CPUExecutionProvider"}
    mod.create_ort_session = create_ort_session
    mod.is_gpu_provider = lambda p: p in REF_GPU
    mod.auto_batch_size = lambda stage, default, provider=None: int(default)
    mod.configure_gpu_addon_paths = lambda: []
    done = install(types.ModuleType("core.asr_engine"), accel_module=mod)
    assert "hardware_accel.create_ort_session" in done
    mod.passed = passed
    return mod


def test_campp_session_through_create_ort_session(accel, tmp_path):
    from write_stage_onnx import write_campp
    from zasr.campp import CamppConfig, synth_weights
    from zasr.hardware_accel import ZASR_PROVIDER
    w = synth_weights(CamppConfig(), int(CAMPP["weight_seed"]))
    path, _ = write_campp(str(tmp_path / "campp-3dspeaker"), w, fused=True)
    sess, info = accel.create_ort_session(None, path, object(), policy="rocm",
                                          stage="CAM++ speaker embedding")
    assert accel.passed == []
    assert info["actual_provider"] == ZASR_PROVIDER and accel.is_gpu_provider(ZASR_PROVIDER)
    assert accel.auto_batch_size("CAM++ speaker embedding", 32, info["actual_provider"]) >= 32
    (warm,) = sess.run(["embs"], {"feats": np.zeros((1, 150, 80), np.float32)})
    assert warm.shape == (1, 192) and np.all(np.isfinite(warm))
    cases = sorted(k[len("emb_in_"):] for k in CAMPP.files if k.startswith("emb_in_"))
    assert cases
    for c in cases:
        got = sess.run(["embs"], {"feats": CAMPP[f"emb_in_{c}"]})[0]
        ref = CAMPP[f"emb_out_{c}"]
        assert got.shape == ref.shape
        mx = float(np.abs(got - ref).max())
        rel = float(np.linalg.norm(got - ref) / np.linalg.norm(ref))
        assert mx <= 2e-3 or rel <= 2e-4, (c, mx, rel)
    sess.engine.close()


def test_vibert_session_through_create_ort_session(accel, tmp_path):
    from write_stage_onnx import write_vibert
    from zasr.hardware_accel import ZASR_PROVIDER
    from zasr.vibert import synth_weights, vibert_base, vibert_tiny
    cases = sorted({k.split("_")[0] for k in VIBERT.files})
    sessions = {}
    for c in cases:
        kind, ws = str(VIBERT[c + "_kind"]), int(VIBERT[c + "_wseed"])
        if (kind, ws) not in sessions:
            cfg = vibert_tiny() if kind == "tiny" else vibert_base()
            d = tmp_path / f"vibert-capu-{kind}-{ws}"
            path, _ = write_vibert(str(d), synth_weights(cfg, ws))
            with open(d / "config.json", "w") as f:
                json.dump({"num_attention_heads": cfg.num_attention_heads}, f)
            sess, info = accel.create_ort_session(None, path, object(), policy="rocm",
                                                  stage="ViBERT punctuation")
            assert accel.is_gpu_provider(info["actual_provider"])  # core/gec_model.py:173
            assert info["actual_provider"] == ZASR_PROVIDER
            sessions[(kind, ws)] = sess
        sess = sessions[(kind, ws)]
        feeds = {k: VIBERT[c + "_" + k] for k in ("input_ids", "attention_mask",
                                                  "token_type_ids", "input_offsets")}
        logits, detect = sess.run(None, feeds)
        for got, ref in ((logits, VIBERT[c + "_logits"]), (detect, VIBERT[c + "_detect_logits"])):
            assert got.shape == ref.shape
            assert float(np.max(np.abs(got - ref))) <= 5e-3
            assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 5e-4
    for s in sessions.values():
        s.engine.close()
    assert accel.passed == []


def test_other_stages_reach_the_reference(accel):
    s, info = accel.create_ort_session(None, "/m/pyannote-onnx/segmentation-community-1.onnx",
                                       object(), policy="rocm", stage="pyannote segmentation")
    assert s == "reference-session" and accel.passed[-1][1] == "pyannote segmentation"
