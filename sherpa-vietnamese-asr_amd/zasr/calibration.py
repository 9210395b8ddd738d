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
from typing import Any, Callable, Dict, List, Optional


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def _gfx_name(version: int) -> str:
    """KFD gfx_target_version (major * 10000 + minor * 100 + stepping) -> "gfxMmS"."""
    major, minor, step = version // 10000, (version // 100) % 100, version % 100
    return f"gfx{major}{minor:x}{step:x}"


def detect_gpus(nodes_dir: str = KFD_NODES) -> List[Dict[str, Any]]:
    """The GPUs the kernel driver reports, asked from the KFD topology (host files only: no
    HIP initialisation): one entry per node with SIMDs, its gfx target and compute units.
    The engine is built for gfx950 only; other targets are listed but not counted as ready."""
    gpus = []
    for d in sorted(glob.glob(os.path.join(nodes_dir, "*")),
                    key=lambda x: int(os.path.basename(x)) if os.path.basename(x).isdigit() else 0):
        props = {}
        try:
            with open(os.path.join(d, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    if v.lstrip("-").isdigit():
                        props[k] = int(v)
        except OSError:
            continue
        if props.get("simd_count", 0) <= 0 or not props.get("gfx_target_version"):
            continue  # a CPU node
        gfx = _gfx_name(props["gfx_target_version"])
        gpus.append({"node": os.path.basename(d), "gfx": gfx, "supported": gfx == "gfx950",
                     "compute_units": props["simd_count"] // max(1, props.get("simd_per_cu", 4)),
                     "name": "AMD Instinct MI355X class (gfx950)" if gfx == "gfx950" else gfx})
    return gpus


def _status() -> Dict[str, Any]:
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib",
                       "libzasr.so")
    gpus = detect_gpus()
    ready = any(g["supported"] for g in gpus) and os.path.exists(lib)
    return {
        "hardware": {"gpus": gpus, "cpu_count": os.cpu_count()},
        "hardware_summary": (f"ASR on {sum(g['supported'] for g in gpus)} gfx950 GPU(s) via "
                             f"libzasr (HIP); {len(gpus)} GPU node(s) reported by KFD"),
        "preferred_provider": "MI355X:HIP",
        "provider_request": "MI355X:HIP",
        "provider_ready": ready,
        "gpu_models_ready": ready,
        "can_optimize": False,
        "reason": "asr_runs_on_mi355x" if ready else (
            "no_gpu" if not gpus else ("no_gfx950_gpu" if not any(g["supported"] for g in gpus)
                                       else "libzasr_missing")),
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
