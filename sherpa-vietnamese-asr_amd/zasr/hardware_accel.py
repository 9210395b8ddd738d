"""Drop-in `core/hardware_accel.py` for the MI355X build.

In the reference this module picks an onnxruntime execution provider (CUDA / DirectML /
OpenVINO / ROCm add-ons) and creates sessions (`core/hardware_accel.py:206-697`).  ASR now
runs in libzasr.so on MI355X and, per the north star, the DirectML/OpenVINO add-on dispatch
is removed.  The names other modules import stay importable (SURVEY §8b:
core/gec_model.py:13, core/speaker_diarization_*.py, core/audio_analyzer.py:155-168,
app.py:30, server_launcher.py:120); ORT session creation raises, since those out-of-scope
stages are not part of this build.
"""
from __future__ import annotations

import glob
import os
from typing import Any, Dict, List, Optional

CPU_PROVIDER = "CPUExecutionProvider"
CUDA_PROVIDER = "CUDAExecutionProvider"
OPENVINO_PROVIDER = "OpenVINOExecutionProvider"
DML_PROVIDER = "DmlExecutionProvider"
ROCM_PROVIDER = "ROCMExecutionProvider"
MI355X_PROVIDER = "MI355X:HIP"


def configure_gpu_addon_paths() -> List[str]:
    """No onnxruntime GPU add-ons in this build."""
    return []


def detect_hardware() -> Dict[str, Any]:
    """MI355X devices visible to this process (KFD render nodes), without touching HIP."""
    nodes = sorted(glob.glob("/dev/dri/renderD*"))
    return {"accelerators": [{"name": "AMD Instinct MI355X (gfx950)", "node": n} for n in nodes],
            "cpu_count": os.cpu_count()}


def best_gpu() -> Optional[Dict[str, Any]]:
    acc = detect_hardware()["accelerators"]
    return acc[0] if acc else None


def is_gpu_provider(provider: Optional[str]) -> bool:
    p = str(provider or "")
    return p not in ("", CPU_PROVIDER, "cpu")


def preferred_gpu_provider(policy: str = "auto", ort_module=None) -> Optional[str]:
    return MI355X_PROVIDER if policy not in ("cpu", "none", "off") else None


def create_ort_session(ort_module, model_path, sess_options=None, policy="cpu", stage="",
                       **kwargs):
    raise RuntimeError(f"onnxruntime sessions are not part of the MI355X build "
                       f"(stage {stage!r}, model {model_path!r}); ASR runs in libzasr.so")


def auto_batch_size(stage: str, default: int, provider: Optional[str] = None) -> int:
    return int(default)


def hardware_summary() -> str:
    acc = detect_hardware()["accelerators"]
    return f"ASR on {len(acc)} MI355X device(s) via libzasr (HIP, gfx950)"
