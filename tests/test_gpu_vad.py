"""Silero VAD on the MI355X through the C ABI vs the fixtures the
reference's own core/vad_utils.py produced (make_golden_vad.py) and vs the oracle.

Tolerance: per-window speech probability within 1e-4 absolute of the reference's (f32 GEMM
and LSTM summation order differ from torch's CPU kernels; the reference publishes no GPU
tolerance for VAD, core/calibration.py:56-61 keeps it on CPU).  Segments must be identical."""
import json
import os

import numpy as np
import pytest

from conftest import gpu_available
from make_golden_vad import case_audio

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "vad_golden.json")))
CASES = {c["name"]: c for c in GOLD["cases"]}
ATOL = 1e-4


@pytest.fixture(scope="module")
def vad_dir(tmp_path_factory):
    if not gpu_available():
        pytest.skip("no GPU")
    from zasr.silero import SileroConfig, save_model_dir, synth_weights
    cfg = SileroConfig()
    return save_model_dir(str(tmp_path_factory.mktemp("silero")), cfg,
                          synth_weights(cfg, GOLD["weights_seed"]))


@pytest.fixture(scope="module")
def sess(vad_dir):
    from zasr.binding import VadSession
    s = VadSession(vad_dir)
    yield s
    s.close()


@pytest.fixture()
def vu(vad_dir, monkeypatch):
    import zasr.vad_utils as vu
    monkeypatch.setenv("ZASR_VAD_MODEL_DIR", vad_dir)
    vu.unload_vad_model()
    yield vu
    vu.unload_vad_model()


def _boost(c):
    return c["fn"] == "get_vad_segments"


@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n]["probs"]))
def test_vad_probs_match_reference(sess, name):
    c = CASES[name]
    p = sess.probs([case_audio(c["audio"])], auto_boost=_boost(c))[0]
    ref = np.array(c["probs"], np.float32)
    assert p.shape == ref.shape
    assert np.max(np.abs(p - ref)) <= ATOL, float(np.max(np.abs(p - ref)))


@pytest.mark.parametrize("name", sorted(CASES))
def test_vad_segments_match_reference(vu, name):
    """zasr.vad_utils (GPU probabilities + host segmentation) returns the reference's result
    and caches probabilities like it."""
    c = CASES[name]
    a = case_audio(c["audio"])
    got = getattr(vu, c["fn"])(a, **c["kwargs"])
    assert [list(s) for s in got] == c["result"]
    cached = vu.get_cached_vad_probs()
    if c["probs"] is None:
        assert cached is None
    else:
        assert np.max(np.abs(cached - np.array(c["probs"], np.float32))) <= ATOL


def test_vad_batch_equals_single_files(vu):
    names = sorted(n for n in CASES if CASES[n]["fn"] == "get_vad_segments")
    audios = [case_audio(CASES[n]["audio"]) for n in names]
    for n, got in zip(names, vu.get_vad_segments_batch(audios)):
        if not CASES[n]["kwargs"]:
            assert [list(s) for s in got] == CASES[n]["result"], n


def test_session_surface_in_reference_loop(sess):
    """The reference's per-window loop (restated in oracle.run_windows) driving the GPU
    session's run(None, feeds) gives the reference's probabilities."""
    from oracle.silero import run_windows
    c = CASES["windows_strict"]
    p = run_windows(sess, case_audio(c["audio"])[:512 * 120])
    ref = np.array(c["probs"][:120], np.float32)
    assert np.max(np.abs(p - ref)) <= ATOL


def test_session_batched_streams(sess):
    """n independent streams in one run() call == n separate calls."""
    rng = np.random.Generator(np.random.PCG64(3))
    x = (rng.normal(size=(5, 576)) * 0.1).astype(np.float32)
    st = (rng.normal(size=(2, 5, 128)) * 0.5).astype(np.float32)
    p, so = sess.run(None, {"input": x, "state": st, "sr": np.array(16000)})
    for i in range(5):
        pi, si = sess.run(None, {"input": x[i:i + 1], "state": st[:, i:i + 1].copy(),
                                 "sr": np.array(16000)})
        assert abs(float(pi[0, 0]) - float(p[i, 0])) <= 1e-6
        np.testing.assert_allclose(si[:, 0], so[:, i], rtol=0, atol=1e-6)


def test_long_file_and_ragged_batch_vs_oracle(sess):
    """10 minutes of speech-like audio (18,750 recurrent steps) plus ragged files in one call,
    against the oracle."""
    from oracle.silero import SileroOracle
    from zasr.silero import SileroConfig, synth_weights
    from zasr.synth_audio import synth_speech
    cfg = SileroConfig()
    orc = SileroOracle(cfg, synth_weights(cfg, GOLD["weights_seed"]))
    audios = [synth_speech(600.0, 41), synth_speech(3.3, 42)[:52_001], np.zeros(100, np.float32),
              synth_speech(9.0, 43) * np.float32(0.01)]
    got = sess.probs(audios, auto_boost=False)
    assert [g.shape[0] for g in got] == [len(a) // 512 for a in audios]
    for a, g in zip(audios, got):
        if len(a) >= 512:
            ref = orc.probs_batched(a)
            assert np.max(np.abs(g - ref)) <= ATOL, float(np.max(np.abs(g - ref)))


def test_parallel_in_time_matches_sequential(vad_dir, monkeypatch):
    """The segmented recurrence (warm-up guesses, state-continuity verification at 1e-6,
    reruns) matches the sequential one-workgroup-per-file probabilities to 1e-5 (two orders
    below the parity tolerance), needs at most 2 passes on speech, and yields the same
    speech segments on the long files."""
    from zasr.binding import VadSession
    from zasr.synth_audio import synth_speech
    audios = [synth_speech(900.0, 51), synth_speech(40.0, 52), synth_speech(300.0, 53) * np.float32(0.02)]
    monkeypatch.setenv("ZASR_VAD_PIT", "0")
    seq = VadSession(vad_dir)
    ref = seq.probs(audios, auto_boost=True)
    assert seq.last_passes == 1
    seq.close()
    monkeypatch.delenv("ZASR_VAD_PIT")
    par = VadSession(vad_dir)
    got = par.probs(audios, auto_boost=True)
    passes = par.last_passes
    par.close()
    worst = max(float(np.max(np.abs(a - b))) for a, b in zip(got, ref))
    assert worst <= 1e-5, worst
    assert passes <= 2, passes
    # the speech segments the reference's get_vad_segments cuts from them (its defaults,
    # core/vad_utils.py:153-260, restated in zasr.vad_utils) are identical
    from zasr.vad_utils import _segments_from_probs
    for a, g, r in zip(audios, got, ref):
        sg = _segments_from_probs(g, len(a), 16000, 0.2, 100, 250, 1000, 250, True)
        sr = _segments_from_probs(r, len(a), 16000, 0.2, 100, 250, 1000, 250, True)
        assert sg == sr
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/vad_pit_passes.json", "w") as f:
        json.dump({"passes": passes, "max_abs_vs_sequential": worst,
                   "windows": [int(x.shape[0]) for x in ref]}, f)
