"""Silero VAD on CPU: the oracle and the host-side segmentation against
the fixtures the reference's own core/vad_utils.py produced (tests/golden/make_golden_vad.py),
and the vectorized segmentation of zasr.vad_utils against the reference's loop."""
import json
import os

import numpy as np
import pytest

from make_golden_vad import case_audio, checksum

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vad_golden.json")))
CASES = {c["name"]: c for c in GOLD["cases"]}


@pytest.fixture(scope="module")
def oracle():
    from oracle.silero import SileroOracle
    from zasr.silero import SileroConfig, synth_weights
    cfg = SileroConfig()
    return SileroOracle(cfg, synth_weights(cfg, GOLD["weights_seed"]))


@pytest.mark.parametrize("name", sorted(CASES))
def test_case_audio_regenerates(name):
    c = CASES[name]
    a = case_audio(c["audio"])
    assert a.shape[0] == c["n_samples"] and checksum(a) == c["sha"]


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_reference_vad(oracle, name):
    """The reference's loop + segmentation restated (oracle.silero) give the reference's
    cached probabilities and segments."""
    from oracle.silero import run_windows, speech_windows, vad_segments
    c = CASES[name]
    a = case_audio(c["audio"])
    sess = oracle.session()
    if c["fn"] == "_run_vad_inference":
        kw = {"threshold": 0.5, "min_silence_ms": 300, "min_speech_ms": 250, **c["kwargs"]}
        p = run_windows(sess, a)
        got = speech_windows(p, kw["threshold"], kw["min_silence_ms"], kw["min_speech_ms"])
    else:
        holder = {}

        def probs_fn(x):
            holder["p"] = run_windows(sess, x)
            return holder["p"]
        got = vad_segments(a, probs_fn, **c["kwargs"])
        p = holder.get("p")
    assert [list(s) for s in got] == c["result"]
    if c["probs"] is None:
        assert p is None
    else:
        np.testing.assert_allclose(p, np.array(c["probs"], np.float32), rtol=0, atol=1e-6)


def test_batched_oracle_matches_sequential(oracle):
    from oracle.silero import run_windows
    a = case_audio(CASES["gappy"]["audio"])
    np.testing.assert_allclose(oracle.probs_batched(a), run_windows(oracle.session(), a),
                               rtol=0, atol=2e-6)


def _settings():
    return [(0.5, 300, 250), (0.2, 100, 250), (0.3, 100, 150), (0.9, 50, 500), (0.5, 0, 0),
            (0.5, 20, 32), (0.1, 1000, 2000)]


@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n]["probs"]))
def test_vectorized_segmentation_matches_reference_loop(name):
    from oracle.silero import speech_windows as loop
    from zasr.vad_utils import speech_windows
    p = np.array(CASES[name]["probs"], np.float32)
    for th, ms_sil, ms_sp in _settings():
        assert speech_windows(p, th, ms_sil, ms_sp) == loop(p, th, ms_sil, ms_sp)


def test_vectorized_segmentation_random_and_edges():
    from oracle.silero import speech_windows as loop
    from zasr.vad_utils import speech_windows
    rng = np.random.Generator(np.random.PCG64(5))
    for trial in range(300):
        n = int(rng.integers(0, 120))
        # blocky sequences so runs and gaps of all lengths occur; exact threshold hits too
        p = np.repeat(rng.choice([0.05, 0.2, 0.3, 0.5, 0.9, 0.95], size=max(1, n // 3)),
                      rng.integers(1, 6, size=max(1, n // 3)))[:n].astype(np.float32)
        for th, ms_sil, ms_sp in _settings():
            assert speech_windows(p, th, ms_sil, ms_sp) == loop(p, th, ms_sil, ms_sp), (trial, th)
    # f64 comparison like the reference's Python floats: f32(0.9) < 0.9
    p = np.full(20, np.float32(0.9))
    assert speech_windows(p, 0.9, 100, 100) == loop(p, 0.9, 100, 100) == []


@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n]["fn"] == "get_vad_segments"
                                        and CASES[n]["probs"]))
def test_host_segments_from_reference_probs(name):
    """zasr.vad_utils's post-processing (retry, fallback, padding, merge) on the reference's
    own probabilities gives the reference's segments."""
    from zasr.vad_utils import _segments_from_probs
    c = CASES[name]
    kw = {"threshold": 0.2, "min_silence_ms": 100, "min_speech_ms": 250, "padding_ms": 1000,
          "merge_gap_ms": 250, "fallback_full": True, **c["kwargs"]}
    got = _segments_from_probs(np.array(c["probs"], np.float32), c["n_samples"], 16000,
                               kw["threshold"], kw["min_silence_ms"], kw["min_speech_ms"],
                               kw["padding_ms"], kw["merge_gap_ms"], kw["fallback_full"])
    assert [list(s) for s in got] == c["result"]


def test_short_audio_needs_no_model(monkeypatch):
    import zasr.vad_utils as vu
    monkeypatch.setattr(vu, "_get_vad_session", lambda: (_ for _ in ()).throw(AssertionError))
    assert vu.get_vad_segments(np.zeros(300, np.float32)) == [(0, 300)]
    assert vu.get_vad_segments(np.zeros(300, np.float32), fallback_full=False) == []
    assert vu._run_vad_inference(np.zeros(511, np.float32)) == []
