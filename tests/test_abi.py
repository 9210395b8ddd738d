"""CPU checks of the drop-in boundary: libzasr.so loads and exports every symbol that
include/zasr.h declares; the host package imports; error paths are reported, not crashed."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "sherpa-vietnamese-asr_amd", "lib", "libzasr.so")
HDR = os.path.join(REPO, "include", "zasr.h")


def header_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(zasr_[a-z0-9_]+)\s*\(", text)))


def test_library_built():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"


def test_exports_match_header():
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    decl = header_functions()
    assert len(decl) >= 20
    missing = [d for d in decl if d not in syms]
    assert not missing, missing


def test_binding_covers_header():
    from zasr.binding import EXPORTS, load_library
    assert sorted(EXPORTS) == header_functions()
    lib = load_library()
    assert lib.zasr_version().startswith(b"zasr")


def test_create_reports_missing_model(tmp_path):
    """zasr_create on a directory without model files fails with a message (no crash).
    (On a GPU-less host this may fail earlier at device selection; both are errors.)"""
    from zasr.binding import Recognizer, ZasrError
    with pytest.raises((FileNotFoundError, ZasrError)):
        Recognizer(str(tmp_path))


def test_drop_in_modules_import():
    import zasr.asr_engine as ae
    import zasr.calibration as cal
    import zasr.hardware_accel as ha
    import zasr.hotword_context as hc
    for name in ("create_recognizer", "compute_fbank_ort", "_ort_beam_search", "decode_chunk",
                 "get_ort", "_log_add", "_compute_token_entropy", "ROVER_MODEL_ID"):
        assert hasattr(ae, name)
    # only configure_gpu_addon_paths is replaced; create_ort_session & co. stay the reference's
    assert ha.configure_gpu_addon_paths() == []
    assert not hasattr(ha, "create_ort_session")
    st = cal.detect_calibration_status()
    assert st["asr"] == "mi355x" and st["preferred_provider"] == "MI355X:HIP"
    calls = []
    rep = cal.run_device_calibration("m", "s", 4, lambda m, p: calls.append(p))
    assert rep["stages"] == {"asr": "mi355x"} and calls == [100]
    with pytest.raises(RuntimeError):
        ae.get_ort()
    assert hc.parse_hotwords_file(os.path.join(REPO, "tests", "golden", "hotword_sample.txt"))


def test_create_recognizer_missing_files(tmp_path):
    import zasr.asr_engine as ae
    with pytest.raises(FileNotFoundError):
        ae.create_recognizer(str(tmp_path))


def test_calibration_asks_the_kfd_topology(tmp_path):
    """zasr.calibration names GPUs from the driver's KFD topology (no HIP call): only gfx950
    nodes count as ready; CPU nodes (no SIMDs) are skipped (ADVICE/VERDICT r03: the status
    must not label every render node an MI355X)."""
    import zasr.calibration as cal
    for node, props in {"0": "cpu_cores_count 64\nsimd_count 0\n",
                        "1": "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n",
                        "2": "simd_count 1216\nsimd_per_cu 4\ngfx_target_version 90402\n"}.items():
        d = tmp_path / node
        d.mkdir()
        (d / "properties").write_text(props)
    gpus = cal.detect_gpus(str(tmp_path))
    assert [(g["node"], g["gfx"], g["supported"], g["compute_units"]) for g in gpus] == \
        [("1", "gfx950", True, 256), ("2", "gfx942", False, 304)]
    assert cal.detect_gpus(str(tmp_path / "missing")) == []
