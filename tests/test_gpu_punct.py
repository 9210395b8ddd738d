"""Punctuation on the MI355X: zasr.punct over the HIP ViBERT session (zasr.binding.
VibertSession) reproduces the reference's own GecBERTModel / restorer output on the fixture
cases whose session is the ViBERT oracle (tests/golden/punct_cases.json, made by running the
reference's handle_batch / restore with tests/golden/make_golden_punct.py): the same text,
and the same feeds for every session run (which chunks each iteration re-ran).  The
fixture's per-case min_margin (smallest gap between the top two adjusted probabilities) is
>= 4e-3, far above the session's f32 logit error."""
import json
import os

import numpy as np
import pytest

from conftest import gpu_available
from punct_sessions import Recorder, write_model_dir

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = [c for c in json.load(open(os.path.join(HERE, "golden", "punct_cases.json"), encoding="utf-8"))
         if c["session"]["kind"] == "oracle"]


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    if not gpu_available():
        pytest.skip("no GPU")
    from zasr.binding import VibertSession
    from zasr.punct import load_word_pieces
    from zasr.vibert import save_model_dir, synth_weights, vibert_tiny
    d = tmp_path_factory.mktemp("punct")
    pieces = load_word_pieces(write_model_dir(str(d / "tok")))
    cfg = vibert_tiny()
    sessions = {}
    for seed in sorted({c["session"]["seed"] for c in CASES}):
        w = synth_weights(cfg, seed)
        w["classifier.weight"] = w["classifier.weight"] * np.float32(40.0)
        sessions[seed] = VibertSession(save_model_dir(str(d / f"v{seed}"), cfg, w))
    yield pieces, sessions
    for s in sessions.values():
        s.close()


@pytest.mark.parametrize("i", range(len(CASES)))
def test_gpu_session_punctuation_equals_reference(env, i):
    from zasr.punct import GecPunctuator
    (tok, start_id, pad_id), sessions = env
    c = CASES[i]
    assert c["min_margin"] >= 4e-3
    rec = Recorder(sessions[c["session"]["seed"]])
    g = GecPunctuator(rec, tok, start_id, pad_id=pad_id)
    if c["kind"] == "restore":
        out = g.restore(c["text"], pause_hints=c["pause_hints"])
    else:
        out = g.handle_batch([t.split() for t in c["texts"]], pause_hints=c["pause_hints"])
    assert rec.calls == c["calls"]
    assert out == c["out"]
