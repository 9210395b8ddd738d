"""Calibration stub (reference `core/calibration.py` is removed per the north star: ASR was
pinned to CPU there, :1369-1374; here it always runs on MI355X).  Keeps the two names the
GUI and web service import (tab_file.py:193-197, web_service/server.py:578-597)."""


def detect_calibration_status():
    return {"status": "not_required", "asr": "mi355x", "calibrated": False,
            "message": "ASR runs on MI355X via libzasr; no provider calibration"}


def run_device_calibration(*args, **kwargs):
    return detect_calibration_status()
