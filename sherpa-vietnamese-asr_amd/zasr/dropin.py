"""Install this build under the reference's module names without editing its source.

    import sys; sys.path.insert(0, "/path/to/reference")          # the reference's tree
    sys.path.insert(0, "/path/to/sherpa-vietnamese-asr_amd")       # this package: zasr only
    import core.asr_engine, core.hardware_accel, core.calibration  # the reference's modules
    from zasr.dropin import install
    install(core.asr_engine, core.hardware_accel, core.calibration)  # before the pipeline runs
    # optional: Silero VAD on the GPU too (reads the reference's
    # models/silero-vad/silero_vad_16k_op15.onnx, or silero_config.json + silero_vad.safetensors)
    import core.vad_utils; install(core.asr_engine, vad_module=core.vad_utils)

This build's modules live in the `zasr` package, so importing them never shadows the
reference's `core` package (both trees can be on sys.path in any order).

What is rebound (the ASR hot path, core/asr_engine.py:698-1326):
  asr_engine      compute_fbank_ort, _log_add, create_recognizer, _ort_beam_search,
                  _compute_token_entropy, _finalize_word_entropy, decode_chunk, and
                  clear_model_cache wrapped so the reference's own version still unloads
                  the punctuation restorer and the diarizer (:743-768); find_silent_regions
                  wrapped (same result: the frame energies run on the GPU, numpy-float32
                  exact, and the signal stays in HBM) so that the chunk plan built from it
                  (:2137-2161) is registered, its batched decode starts at once for the
                  loaded recognizers, and the per-chunk decode_chunk calls of the two
                  workers are served from that ONE decode (zasr.asr_engine, plan-ahead)
  hardware_accel  configure_gpu_addon_paths (the DirectML / OpenVINO add-on dispatch is
                  removed per the north star); create_ort_session, is_gpu_provider and
                  auto_batch_size wrapped: the "CAM++ speaker embedding" and "ViBERT
                  punctuation" sessions (core/speaker_diarization_senko_campp_optimized.py:
                  364-368, core/gec_model.py:168-172) are libzasr.so engines with the
                  onnxruntime run() surface their callers use; every other stage (pyannote,
                  DNSMOS, ...) gets the reference's own onnxruntime session
  calibration     detect_calibration_status / run_device_calibration (the provider picker is
                  removed per the north star; ASR always runs on MI355X)
  vad_utils       (only when vad_module is given) _get_vad_session, unload_vad_model,
                  get_cached_vad_probs, _run_vad_inference, get_vad_segments; and the
                  get_vad_segments / unload_vad_model names asr_engine imported from it
                  (core/asr_engine.py:580)

get_ort, TranscriberPipeline, the overlap merge, ROVER vote and UI glue stay the
reference's.  create_recognizer reads the hotword file and score through the reference
module's own get_hotwords_config (core/config.py:385-408), as the reference does (:993-1003).
Returns the list of names rebound.
"""
from __future__ import annotations

import sys
from types import ModuleType
from typing import List, Optional

ENGINE_NAMES = ("compute_fbank_ort", "_log_add", "create_recognizer", "_ort_beam_search",
                "_compute_token_entropy", "_finalize_word_entropy", "decode_chunk")
ACCEL_NAMES = ("configure_gpu_addon_paths",)
WRAPPED_ACCEL = {"create_ort_session": "make_create_ort_session",
                 "is_gpu_provider": "make_is_gpu_provider",
                 "auto_batch_size": "make_auto_batch_size"}
CALIBRATION_NAMES = ("detect_calibration_status", "run_device_calibration")
VAD_NAMES = ("_get_vad_session", "unload_vad_model", "get_cached_vad_probs",
             "_run_vad_inference", "get_vad_segments")
VAD_ENGINE_NAMES = ("get_vad_segments", "unload_vad_model")


def _caller_uses_wpe(frame) -> bool:
    """True when the planner's caller is a TranscriberPipeline whose config enables WPE
    dereverberation (core/asr_engine.py:2248): its `self.config["preprocess_wpe"]`."""
    try:
        cfg = getattr(frame.f_locals.get("self"), "config", None)
        return bool(cfg.get("preprocess_wpe", False)) if hasattr(cfg, "get") else False
    except Exception:
        return False


def install(engine_module: ModuleType, accel_module: Optional[ModuleType] = None,
            calibration_module: Optional[ModuleType] = None,
            vad_module: Optional[ModuleType] = None) -> List[str]:
    from zasr import asr_engine as ours
    from zasr import calibration as ours_cal
    from zasr import hardware_accel as ours_hw
    if engine_module is ours:
        raise ValueError("install() needs the reference's core.asr_engine module, got zasr's own")
    done = []
    for n in ENGINE_NAMES:
        setattr(engine_module, n, getattr(ours, n))
        done.append("asr_engine." + n)
    orig_clear = getattr(engine_module, "clear_model_cache", None)
    if orig_clear is not None and not getattr(orig_clear, "_zasr_wrapped", False):
        def clear_model_cache(which="all"):
            ours.clear_model_cache(which)
            return orig_clear(which)
        clear_model_cache._zasr_wrapped = True
        clear_model_cache.__doc__ = orig_clear.__doc__
        engine_module.clear_model_cache = clear_model_cache
        done.append("asr_engine.clear_model_cache")
    orig_fsr = getattr(engine_module, "find_silent_regions", None)
    if orig_fsr is not None and not getattr(orig_fsr, "_zasr_wrapped", False):
        split_fn = getattr(engine_module, "find_best_split_point", None)

        def find_silent_regions(audio_data, *args, **kwargs):
            # with preprocess_wpe the workers decode WPE-processed copies, never views of the
            # planned signal (:2248, :2338-2341): register the plan, start no decode for it
            start = not _caller_uses_wpe(sys._getframe(1))
            if not args and not kwargs:  # the planner's calls (:2139, :2183) use the defaults
                try:  # the GPU silence detector: same regions, plan registered + decoding
                    regions = ours.plan_ahead_regions(audio_data, split_fn, start=start)
                    if regions is not None:
                        return regions
                except Exception as e:  # routing is an optimisation: never break the caller
                    ours.logger.warning(f"[zasr] GPU planner skipped: {e}")
            regions = orig_fsr(audio_data, *args, **kwargs)
            if not args and not kwargs:
                try:
                    ours.register_plan_from_regions(audio_data, regions, split_fn, start=start)
                except Exception as e:
                    ours.logger.warning(f"[zasr] plan registration skipped: {e}")
            return regions
        find_silent_regions._zasr_wrapped = True
        find_silent_regions.__doc__ = orig_fsr.__doc__
        engine_module.find_silent_regions = find_silent_regions
        done.append("asr_engine.find_silent_regions")
    ours.set_host_module(engine_module)
    if accel_module is not None:
        for n in ACCEL_NAMES:
            setattr(accel_module, n, getattr(ours_hw, n))
            done.append("hardware_accel." + n)
        # CAM++ / ViBERT sessions from libzasr.so, everything else the reference's own
        for n, make in WRAPPED_ACCEL.items():
            orig = getattr(accel_module, n, None)
            if orig is not None and not getattr(orig, "_zasr_wrapped", False):
                setattr(accel_module, n, getattr(ours_hw, make)(orig))
                done.append("hardware_accel." + n)
    if calibration_module is not None:
        for n in CALIBRATION_NAMES:
            setattr(calibration_module, n, getattr(ours_cal, n))
            done.append("calibration." + n)
    if vad_module is not None:
        from zasr import vad_utils as ours_vad
        if vad_module is ours_vad:
            raise ValueError("install() needs the reference's core.vad_utils module")
        ours_vad.set_base_dir(getattr(vad_module, "BASE_DIR", None))
        for n in VAD_NAMES:
            setattr(vad_module, n, getattr(ours_vad, n))
            done.append("vad_utils." + n)
        for n in VAD_ENGINE_NAMES:
            if hasattr(engine_module, n):
                setattr(engine_module, n, getattr(ours_vad, n))
                done.append("asr_engine." + n)
    return done
