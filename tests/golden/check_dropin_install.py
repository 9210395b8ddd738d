"""Build-container check that zasr.dropin.install really rebinds the REFERENCE's modules.

Run here only (the reference never travels to the GPU box):

    python tests/golden/check_dropin_install.py [/root/reference]

It puts the reference tree and this build's package on sys.path together (reference first,
then ours, then the other order in a second process), imports the reference's own
`core.asr_engine`, `core.hardware_accel` and `core.calibration`, runs install(), and asserts:
  * the hot-path names of the reference module object are now this build's functions;
  * the names this build must NOT take over (get_ort, TranscriberPipeline, rover_merge_words,
    merge_chunks_with_overlap) are still the reference's; create_ort_session, is_gpu_provider
    and auto_batch_size are wrapped: the reference's own diarizer initialize() gets its CAM++
    session from libzasr.so (its pyannote session stays onnxruntime's), the ViBERT stage
    likewise, and the reference's provider checks accept it (check_session_routing);
  * clear_model_cache is wrapped: this build's cache is dropped AND the reference's own
    function still runs (it unloads the punctuation restorer / diarizer);
  * create_recognizer's hotword route goes through the reference's get_hotwords_config
    (core/config.py:385-408): the file it prepares from the reference's hotword.txt and its
    score 1.5 are what this build uses.
  * the reference's own, unchanged TranscriberPipeline (core/asr_engine.py:1877-3459) run
    over the installed build -- planner, two worker threads calling decode_chunk per chunk
    (:2219-2237, :2326-2397), timestamp map, overlap merge -- reaches the engine as ONE
    batched decode of the whole chunk plan (plan-ahead route), with segments identical to
    the per-chunk route (ZASR_PLAN_AHEAD=0).  The engine is a deterministic CPU stand-in
    (tests/test_dropin_plan.py FakeHandle; no GPU here); the audio loader is replaced by a
    function returning synthetic speech (soundfile / ffmpeg are absent; audio I/O is outside
    the path), and the pipeline's phase file is redirected to the temp dir.
Prints "dropin install ok" and "pipeline dispatch ok" and exits 0 on success.
"""
from __future__ import annotations

import contextlib
import io
import os
import subprocess
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(os.path.dirname(os.path.dirname(HERE)), "sherpa-vietnamese-asr_amd")


def check(ref_root: str, ours_first: bool) -> None:
    paths = [PKG, ref_root] if ours_first else [ref_root, PKG]
    for p in reversed(paths):
        sys.path.insert(0, p)
    with contextlib.redirect_stdout(io.StringIO()):
        import core.asr_engine as ref
        import core.calibration as ref_cal
        import core.hardware_accel as ref_hw
    assert os.path.realpath(ref.__file__).startswith(os.path.realpath(ref_root)), ref.__file__
    import zasr.asr_engine as ours
    import zasr.calibration as ours_cal
    import zasr.hardware_accel as ours_hw
    from zasr.dropin import ACCEL_NAMES, CALIBRATION_NAMES, ENGINE_NAMES, install

    keep = {n: getattr(ref, n) for n in ("get_ort", "TranscriberPipeline", "rover_merge_words",
                                          "merge_chunks_with_overlap")}
    orig_hw = {n: getattr(ref_hw, n) for n in ("create_ort_session", "is_gpu_provider",
                                                "auto_batch_size")}
    orig_clear = ref.clear_model_cache
    done = install(ref, ref_hw, ref_cal)

    for n in ENGINE_NAMES:
        assert getattr(ref, n) is getattr(ours, n), n
    for n in ACCEL_NAMES:
        assert getattr(ref_hw, n) is getattr(ours_hw, n), n
    for n in CALIBRATION_NAMES:
        assert getattr(ref_cal, n) is getattr(ours_cal, n), n
    for n, f in keep.items():
        assert getattr(ref, n) is f, n
    for n, f in orig_hw.items():  # wrapped, not replaced: other stages reach the reference's
        assert getattr(ref_hw, n) is not f and getattr(ref_hw, n)._zasr_wrapped, n
    assert "asr_engine.create_recognizer" in done and "asr_engine.decode_chunk" in done
    check_session_routing(ref_root, ref_hw, ours_hw, orig_hw)

    # clear_model_cache: ours drops its cache, the reference's still runs
    assert ref.clear_model_cache is not orig_clear
    ours._recognizer_cache[("sentinel",)] = {"handle": None}
    calls = []
    real = orig_clear

    def spy(which="all"):
        calls.append(which)
        return real(which)
    # re-install over a spy to observe the call-through without touching the module's state
    ref.clear_model_cache = spy
    install(ref)
    with contextlib.redirect_stdout(io.StringIO()):
        ref.clear_model_cache("all")
    assert calls == ["all"], calls
    assert not ours._recognizer_cache

    # hotword route: the reference's get_hotwords_config decides file and score
    model_dir = os.path.join(ref_root, "models")  # bpe.model absent: the config still resolves
    with contextlib.redirect_stdout(io.StringIO()):
        hw_file, hw_score = ours._hotword_config(model_dir)
    assert hw_file and os.path.exists(hw_file), hw_file
    assert hw_score == 1.5, hw_score
    from zasr.hotword_context import parse_hotwords_file
    phrases = parse_hotwords_file(hw_file)
    assert len(phrases) > 200, len(phrases)
    os.remove(hw_file)  # prepare_hotwords_file writes a temp copy

    # VAD (opt-in): the reference's core.vad_utils names and the two asr_engine imported
    # from it (core/asr_engine.py:580) become this build's; BASE_DIR decides the model dir
    with contextlib.redirect_stdout(io.StringIO()):
        import core.vad_utils as ref_vad
    import zasr.vad_utils as ours_vad
    from zasr.dropin import VAD_ENGINE_NAMES, VAD_NAMES
    done_vad = install(ref, vad_module=ref_vad)
    for n in VAD_NAMES:
        assert getattr(ref_vad, n) is getattr(ours_vad, n), n
    for n in VAD_ENGINE_NAMES:
        assert getattr(ref, n) is getattr(ours_vad, n), n
    os.environ.pop("ZASR_VAD_MODEL_DIR", None)
    assert ours_vad.model_dir() == os.path.join(ref_vad.BASE_DIR, "models", "silero-vad")
    done += [d for d in done_vad if d.startswith("vad_utils.")]
    print("dropin install ok (%s first): %d names rebound, %d hotword phrases via "
          "get_hotwords_config" % ("zasr" if ours_first else "reference", len(done), len(phrases)))


def check_session_routing(ref_root, ref_hw, ours_hw, orig_hw) -> None:
    """The reference's own diarizer initialize() (core/speaker_diarization_senko_campp_
    optimized.py:344-398) and GecBERTModel's session call (core/gec_model.py:168-191) over the
    installed factory: CAM++ / ViBERT sessions are libzasr.so engines (a recording stand-in
    here: no GPU in this container), the pyannote segmentation session the diarizer builds
    directly stays onnxruntime's, and the reference's provider checks accept the engine.
    onnxruntime is absent here: a recording stand-in module takes its place."""
    made, ort_made = [], []

    class Standin:
        def __init__(self, model_path, device_id=0):
            made.append(model_path)
            self.calls = []

        def run(self, names, feeds):
            self.calls.append((names, {k: np.asarray(v).shape for k, v in feeds.items()}))
            n = np.asarray(feeds["feats"]).shape[0]
            return [np.ones((n, 192), np.float32)]

    class FakeOrt(types.ModuleType):
        class SessionOptions:
            pass

        class GraphOptimizationLevel:
            ORT_ENABLE_ALL = 99

        class ExecutionMode:
            ORT_SEQUENTIAL = 0

        @staticmethod
        def set_default_logger_severity(level):
            pass

        @staticmethod
        def get_available_providers():
            return ["CPUExecutionProvider"]

        @staticmethod
        def InferenceSession(path, opts=None, providers=None):
            ort_made.append((path, providers))
            return types.SimpleNamespace(get_providers=lambda: ["CPUExecutionProvider"])

    saved = (ours_hw.CamppOrtSession, ours_hw.VibertOrtSession, sys.modules.get("onnxruntime"))
    ours_hw.CamppOrtSession = ours_hw.VibertOrtSession = Standin
    sys.modules["onnxruntime"] = FakeOrt("onnxruntime")
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            from core.speaker_diarization_senko_campp_optimized import SenkoCamppDiarizerOptimized
            dz = SenkoCamppDiarizerOptimized(model_dir="/models/campp-3dspeaker",
                                             execution_provider="rocm")
            dz.initialize()
        assert made == ["/models/campp-3dspeaker/campplus_cn_en_common_200k.onnx"], made
        assert dz.emb_sess.calls == [(["embs"], {"feats": (1, 150, 80)})], dz.emb_sess.calls
        assert dz.batch_size == ours_hw.CAMPP_BATCH, dz.batch_size
        assert [p for p, _ in ort_made] == [dz.seg_path], ort_made  # segmentation: onnxruntime
        vib = os.path.join("/models/vibert-capu", "vibert-capu.onnx")
        sess, info = ref_hw.create_ort_session(sys.modules["onnxruntime"], vib, object(),
                                               policy="rocm", stage="ViBERT punctuation")
        assert made[-1] == vib and ref_hw.is_gpu_provider(info.get("actual_provider"))
        assert ref_hw.auto_batch_size("ViBERT punctuation", 32,
                                      info["actual_provider"]) == ours_hw.VIBERT_BATCH
        # the reference's own functions still answer for their providers
        assert ref_hw.is_gpu_provider("ROCMExecutionProvider") == orig_hw["is_gpu_provider"](
            "ROCMExecutionProvider")
        assert ref_hw.auto_batch_size("DNSMOS", 8, "CPUExecutionProvider") == 8
    finally:
        ours_hw.CamppOrtSession, ours_hw.VibertOrtSession = saved[:2]
        if saved[2] is None:
            sys.modules.pop("onnxruntime", None)
        else:
            sys.modules["onnxruntime"] = saved[2]


def check_pipeline(ref_root: str) -> None:
    import tempfile

    import numpy as np
    sys.path[:0] = [ref_root, PKG, os.path.dirname(HERE)]
    with contextlib.redirect_stdout(io.StringIO()):
        import core.asr_engine as ref
        import core.calibration as ref_cal
        import core.hardware_accel as ref_hw
    from test_dropin_plan import FakeHandle
    from zasr import asr_engine as ours
    from zasr.dropin import install
    from zasr.synth_audio import synth_speech
    install(ref, ref_hw, ref_cal)
    ref.TranscriberPipeline._phase_file = os.path.join(tempfile.gettempdir(), "zasr_asr_phase")
    audio = synth_speech(300.0, 5)
    ref.load_audio = lambda *a, **k: audio.copy()
    handle = {}

    class StandIn:  # the Recognizer surface decode_chunk / compute_fbank_ort use
        def __init__(self, *a, **k):
            self.vocab_size = 64

        def decode(self, chunks, beam=0):
            return handle["h"].decode(chunks, beam)

        def decode_features(self, feats, beam=0):
            return handle["h"].decode_features(feats, beam)

        def fbank(self, a):
            return handle["h"].fbank(a)
    ours.Recognizer = StandIn
    md = tempfile.mkdtemp(prefix="zasr_dropin_model_")
    for f in ("config.json", "model.safetensors"):
        with open(os.path.join(md, f), "w") as fh:
            fh.write("{}")
    toks = ["<blk>", "<sos/eos>", "<unk>"] + [f"\u2581w{i}" if i % 3 == 0 else f"p{i}"
                                             for i in range(3, 64)]
    with open(os.path.join(md, "tokens.txt"), "w", encoding="utf-8") as fh:
        fh.write("".join(f"{t} {i}\n" for i, t in enumerate(toks)))
    cfg = {"cpu_threads": 4, "bypass_vad": True, "speaker_diarization": False,
           "restore_punctuation": False, "skip_preprocessing": True}
    runs = {}
    for route in ("1", "0"):
        os.environ["ZASR_PLAN_AHEAD"] = route
        ours.clear_model_cache()
        handle["h"] = FakeHandle()
        with contextlib.redirect_stdout(io.StringIO()) as out:
            res = ref.TranscriberPipeline("synthetic.wav", md, cfg).run()
        runs[route] = (handle["h"].calls, res, out.getvalue())
    calls, res, log = runs["1"]
    per_calls, per_res, _ = runs["0"]
    n_chunks = len(per_calls)
    assert n_chunks >= 4 and per_calls == [1] * n_chunks, per_calls  # the 2-worker path ran
    assert calls == [n_chunks], (calls, log[-2000:])
    strip = lambda r: [{k: v for k, v in seg.items()} for seg in r["segments"]]  # noqa: E731
    assert strip(res) == strip(per_res)
    assert len(res["segments"]) > 10
    os.environ.pop("ZASR_PLAN_AHEAD", None)
    print("pipeline dispatch ok: the reference's TranscriberPipeline made %d decode_chunk calls "
          "from 2 workers, served by %d batched decode call(s) of %d chunks; %d segments equal "
          "to the per-chunk route" % (n_chunks, len(calls), calls[0], len(res["segments"])))


def main():
    ref_root = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "/root/reference"
    if "--ours-first" in sys.argv:
        check(ref_root, True)
        return
    if "--ref-first" in sys.argv:
        check(ref_root, False)
        return
    if "--pipeline" in sys.argv:
        check_pipeline(ref_root)
        return
    for flag in ("--ref-first", "--ours-first", "--pipeline"):  # fresh interpreter each
        r = subprocess.run([sys.executable, os.path.abspath(__file__), ref_root, flag],
                           capture_output=True, text=True)
        sys.stdout.write(r.stdout)
        if r.returncode != 0:
            sys.stderr.write(r.stderr)
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
