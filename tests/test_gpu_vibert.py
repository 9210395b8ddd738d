"""ViBERT-capu on the MI355X through the C ABI vs the fixtures the
reference's own Seq2LabelsModel produced and vs the oracle on a full mini-batch.

Tolerance: the reference's acceptance rule for a GPU ViBERT (core/calibration.py:95-101,
1279-1286): max_abs <= 5e-3 or rel_l2 <= 5e-4 -- held here as both."""
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "vibert_golden.npz"))
CASES = sorted({k.split("_")[0] for k in GOLD.files})


@pytest.fixture(scope="module")
def sessions(tmp_path_factory):
    if not gpu_available():
        pytest.skip("no GPU")
    from zasr.binding import VibertSession
    from zasr.vibert import save_model_dir, synth_weights, vibert_base, vibert_tiny
    out = {}
    for c in CASES:
        kind, ws = str(GOLD[c + "_kind"]), int(GOLD[c + "_wseed"])
        if (kind, ws) in out:
            continue
        cfg = vibert_tiny() if kind == "tiny" else vibert_base()
        w = synth_weights(cfg, ws)
        d = str(tmp_path_factory.mktemp(f"vibert_{kind}"))
        save_model_dir(d, cfg, w)
        out[(kind, ws)] = (cfg, w, VibertSession(d))
    yield out
    for _, _, s in out.values():
        s.close()


def _check(got, ref):
    assert got.shape == ref.shape
    assert np.max(np.abs(got - ref)) <= 5e-3, float(np.max(np.abs(got - ref)))
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) <= 5e-4


@pytest.mark.parametrize("c", CASES)
def test_vibert_matches_reference(sessions, c):
    cfg, w, sess = sessions[(str(GOLD[c + "_kind"]), int(GOLD[c + "_wseed"]))]
    feeds = {k: GOLD[c + "_" + k] for k in ("input_ids", "attention_mask", "token_type_ids",
                                            "input_offsets")}
    lg, dl = sess.run(None, feeds)
    _check(lg, GOLD[c + "_logits"])
    _check(dl, GOLD[c + "_detect_logits"])


def test_vibert_base_full_minibatch_matches_oracle(sessions):
    """The reference's mini-batch (32 sentences of up to 64 words) at the real ViBERT-base
    shape."""
    from make_golden_vibert import make_inputs
    from oracle.vibert import VibertOracle
    key = [k for k in sessions if k[0] == "base"][0]
    cfg, w, sess = sessions[key]
    ids, am, tt, off = make_inputs(cfg, 32, 40, 777)
    lg, dl = sess.run(["logits", "detect_logits"], {"input_ids": ids, "attention_mask": am,
                                                    "token_type_ids": tt, "input_offsets": off})
    rl, rd = VibertOracle(cfg, w).run(ids, am, tt, off)
    _check(lg, rl)
    _check(dl, rd)


def test_vibert_rejects_out_of_range_ids(sessions):
    """input_ids / token_type_ids outside the embedding tables are an error (onnxruntime's
    Gather raises; the device gather would read out of bounds), checked before any copy."""
    from zasr.binding import ZasrError
    cfg, w, sess = next(iter(sessions.values()))
    c = CASES[0]
    feeds = {k: np.array(GOLD[c + "_" + k]) for k in ("input_ids", "attention_mask",
                                                      "token_type_ids", "input_offsets")}
    for key, bad in (("input_ids", cfg.vocab_size), ("input_ids", -1),
                     ("token_type_ids", cfg.type_vocab_size)):
        f = {k: v.copy() for k, v in feeds.items()}
        f[key][0, 1] = bad
        with pytest.raises(ZasrError, match="out of range"):
            sess.run(None, f)
    sess.run(None, feeds)  # the session stays usable
