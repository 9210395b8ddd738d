"""CAM++ oracle (oracle/campplus.py) vs the reference's own outputs.

tests/golden/make_golden_campp.py ran the reference's CAMPPlus class (convert_onnx/
export_campplus_onnx.py) and _compute_fbank_vectorized (core/speaker_diarization_senko_campp_
optimized.py:86-159, mel matrix injected: kaldi_native_fbank is absent) on seeded inputs."""
import os

import numpy as np
import pytest

from oracle.campplus import CamppOracle, campp_fbank
from zasr.campp import CamppConfig, campp_flops, param_shapes, synth_weights, window_plan

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "campp_golden.npz"))
EMB_CASES = sorted(k[len("emb_in_"):] for k in GOLD.files if k.startswith("emb_in_"))


@pytest.fixture(scope="module")
def orc():
    cfg = CamppConfig()
    return CamppOracle(cfg, synth_weights(cfg, int(GOLD["weight_seed"])))


@pytest.mark.parametrize("case", EMB_CASES)
def test_oracle_embedding_matches_reference(orc, case):
    got = orc.embed(GOLD[f"emb_in_{case}"])
    ref = GOLD[f"emb_out_{case}"]
    # the reference's own acceptance rule for CAM++ outputs (core/calibration.py:71-78,
    # 1279-1286): max_abs <= 2e-3 OR rel_l2 <= 2e-4.  Random-weight embeddings reach |x| ~ 50,
    # so rel_l2 is the binding test (it must hold on every case)
    rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    assert rel <= 2e-4, (rel, float(np.max(np.abs(got - ref))))


@pytest.mark.parametrize("i", range(4))
def test_oracle_fbank_matches_reference(i):
    got = campp_fbank(GOLD[f"fb_in_{i}"])
    ref = GOLD[f"fb_out_{i}"]
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5)


def test_param_count_and_window_plan():
    assert sum(int(np.prod(s)) for s in param_shapes(CamppConfig()).values()) == 6930720
    assert window_plan(9) == []
    assert window_plan(97) == [(0, 97)]
    assert window_plan(150) == [(0, 150)]  # pos + window < n is false at once: tail only
    assert window_plan(211) == [(0, 150), (60, 150), (61, 150)]
    assert window_plan(300)[-1] == (150, 150)
    assert campp_flops(CamppConfig(), 150) > 1e8
