"""The `core/calibration.py` names the GUI and the web service import
(`tab_file.py:193-208`, `web_service/server.py:578-606`).

The reference's calibration benchmarks every stage on CPU and on an onnxruntime GPU provider
and picks one per stage, with ASR pinned to CPU (`core/calibration.py:1369-1374`).  Per the
north star the picker is removed: ASR always runs in libzasr on MI355X.  These two functions
keep the callers working with the reference's report shape (`:274-316`): the status says there
is nothing to calibrate and why.
"""
from __future__ import annotations

import glob
import os
from typing import Any, Callable, Dict, Optional


def _status() -> Dict[str, Any]:
    nodes = sorted(glob.glob("/dev/dri/renderD*"))
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                       "libzasr.so")
    gpus = [{"name": "AMD Instinct MI355X (gfx950)", "node": n} for n in nodes]
    ready = bool(gpus) and os.path.exists(lib)
    return {
        "hardware": {"gpus": gpus, "cpu_count": os.cpu_count()},
        "hardware_summary": f"ASR on {len(gpus)} GPU node(s) via libzasr (HIP, gfx950)",
        "preferred_provider": "MI355X:HIP",
        "provider_request": "MI355X:HIP",
        "provider_ready": ready,
        "gpu_models_ready": ready,
        "can_optimize": False,
        "reason": "asr_runs_on_mi355x" if ready else ("no_gpu" if not gpus else "libzasr_missing"),
        "recommended_addon": None,
        "recommended_gpu_models": {"installed": ready},
        "installed_addons": [],
        "light_probe": [],
        "asr": "mi355x",
        "calibrated": False,
    }


def detect_calibration_status() -> Dict[str, Any]:
    """`core/calibration.py:274` report keys; nothing to calibrate (no provider choice)."""
    return _status()


def run_device_calibration(model_name: Optional[str] = None, speaker_model: Optional[str] = None,
                           cpu_threads: Optional[int] = None,
                           callback: Optional[Callable[[str, int], None]] = None,
                           *args, **kwargs) -> Dict[str, Any]:
    """`core/calibration.py:1525`: reports the fixed placement instead of benchmarking
    providers (the stage choice it would make is the one already in effect)."""
    if callback is not None:
        callback("ASR runs on MI355X via libzasr: no calibration needed", 100)
    report = _status()
    report.update({"model": model_name, "speaker_model": speaker_model,
                   "cpu_threads": cpu_threads, "stages": {"asr": "mi355x"}})
    return report
