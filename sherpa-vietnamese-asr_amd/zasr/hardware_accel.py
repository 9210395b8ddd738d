"""The `core/hardware_accel.py` name this build replaces.

The reference module picks an onnxruntime execution provider and creates sessions for every
stage (`core/hardware_accel.py:206-697`).  ASR no longer uses onnxruntime (it runs in
libzasr.so), and per the north star the DirectML / OpenVINO add-on DLL dispatch is removed:
zasr.dropin.install() rebinds only `configure_gpu_addon_paths` (below).  Everything else --
create_ort_session, is_gpu_provider, auto_batch_size, the provider pickers -- stays the
reference's own, so the stages outside the ASR path (diarization, punctuation, DNSMOS) keep
creating their onnxruntime sessions exactly as before.
"""
from __future__ import annotations

from typing import List


def configure_gpu_addon_paths() -> List[str]:
    """The reference adds the DirectML / OpenVINO / CUDA add-on directories to the DLL search
    path and returns them (`core/hardware_accel.py:60-118`); that dispatch is removed, so there
    are none."""
    return []
