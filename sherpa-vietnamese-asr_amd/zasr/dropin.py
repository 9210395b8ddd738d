"""Install this build under the reference's module names without editing its source.

    import core.asr_engine, core.hardware_accel           # the reference's modules
    from zasr.dropin import install
    install(core.asr_engine, core.hardware_accel)          # before TranscriberPipeline runs

Every hot-path entry point of the reference module is rebound to the HIP implementation
(core/asr_engine.py:686-1326 + core/hardware_accel.py), so the reference's own
TranscriberPipeline, overlap merge and ROVER vote run unchanged on top of libzasr.  Names the
reference defines but this build does not replace (pipeline, merges, VAD, UI glue) are left
alone.  Returns the list of names rebound.
"""
from __future__ import annotations

from types import ModuleType
from typing import List, Optional

ENGINE_NAMES = ("get_ort", "compute_fbank_ort", "_log_add", "clear_model_cache",
                "create_recognizer", "_ort_beam_search", "_compute_token_entropy",
                "_finalize_word_entropy", "decode_chunk", "ROVER_MODEL_IDS", "ROVER_MODEL_ID")
ACCEL_NAMES = ("configure_gpu_addon_paths", "detect_hardware", "is_gpu_provider",
               "create_ort_session", "auto_batch_size", "hardware_summary")


def install(engine_module: ModuleType, accel_module: Optional[ModuleType] = None) -> List[str]:
    from core import asr_engine as ours
    from core import hardware_accel as ours_hw
    done = []
    for n in ENGINE_NAMES:
        if hasattr(ours, n):
            setattr(engine_module, n, getattr(ours, n))
            done.append("asr_engine." + n)
    if accel_module is not None:
        for n in ACCEL_NAMES:
            if hasattr(ours_hw, n):
                setattr(accel_module, n, getattr(ours_hw, n))
                done.append("hardware_accel." + n)
    return done
