"""ViBERT oracle (oracle/vibert.py) vs the reference's own Seq2LabelsModel outputs
(tests/golden/make_golden_vibert.py).  Tolerance: the reference's ViBERT
acceptance rule (core/calibration.py:95-101, 1279-1286): max_abs <= 5e-3 or rel_l2 <= 5e-4;
the restatement is held to both."""
import os

import numpy as np
import pytest

from oracle.vibert import VibertOracle
from zasr.vibert import param_shapes, synth_weights, vibert_base, vibert_tiny

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "vibert_golden.npz"))
CASES = sorted({k.split("_")[0] for k in GOLD.files})


def _case(c):
    kind = str(GOLD[c + "_kind"])
    cfg = vibert_tiny() if kind == "tiny" else vibert_base()
    return cfg, synth_weights(cfg, int(GOLD[c + "_wseed"]))


@pytest.mark.parametrize("c", CASES)
def test_vibert_oracle_matches_reference(c):
    cfg, w = _case(c)
    lg, dl = VibertOracle(cfg, w).run(GOLD[c + "_input_ids"], GOLD[c + "_attention_mask"],
                                      GOLD[c + "_token_type_ids"], GOLD[c + "_input_offsets"])
    for got, ref in ((lg, GOLD[c + "_logits"]), (dl, GOLD[c + "_detect_logits"])):
        assert got.shape == ref.shape
        assert np.max(np.abs(got - ref)) <= 5e-3
        assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 5e-4


def test_vibert_base_param_count():
    n = sum(int(np.prod(s)) for s in param_shapes(vibert_base()).values())
    assert 110e6 < n < 120e6, n
