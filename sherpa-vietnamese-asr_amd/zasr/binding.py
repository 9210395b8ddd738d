"""ctypes binding of libzasr.so (include/zasr.h).

This is the thin host layer the drop-in `core/asr_engine.py` sits on.  There is no CPU
fallback: if the shared library is missing or fails to load, construction raises.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
from typing import List, Optional, Sequence

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_LIB = os.path.join(_PKG, "lib", "libzasr.so")

# every symbol declared in include/zasr.h (the CPU test checks the .so exports them all)
EXPORTS = (
    "zasr_create", "zasr_destroy", "zasr_convert_model", "zasr_convert_stage_model", "zasr_fbank", "zasr_decode_batch", "zasr_decode_features",
    "zasr_decode_device", "zasr_decode_device_batches", "zasr_encode_features", "zasr_search_encoder_out",
    "zasr_result_count", "zasr_result_num_tokens", "zasr_result_num_frames",
    "zasr_result_tokens", "zasr_result_frames", "zasr_result_log_probs",
    "zasr_result_token_stats", "zasr_result_free", "zasr_vocab_size", "zasr_joiner_dim",
    "zasr_profile_enable", "zasr_profile_reset", "zasr_profile_report", "zasr_last_error",
    "zasr_version", "zasr_campp_create", "zasr_campp_destroy", "zasr_campp_embedding_dim",
    "zasr_campp_fbank", "zasr_campp_embed", "zasr_campp_embed_device", "zasr_campp_windows_device",
    "zasr_vibert_create", "zasr_vibert_destroy", "zasr_vibert_num_labels",
    "zasr_vibert_num_detect", "zasr_vibert_run",
    "zasr_vad_create", "zasr_vad_destroy", "zasr_vad_probs", "zasr_vad_probs_device",
    "zasr_vad_window", "zasr_vad_last_passes", "zasr_silence_flags",
    "zasr_create_stream", "zasr_destroy_stream", "zasr_stream_accept_waveform",
    "zasr_decode_stream", "zasr_decode_streams", "zasr_stream_is_decoded",
    "zasr_stream_num_tokens", "zasr_stream_num_frames", "zasr_stream_tokens",
    "zasr_stream_frames", "zasr_stream_log_probs", "zasr_stream_token_stats",
    "zasr_stream_result_json", "zasr_set_tokens", "zasr_model_routes",
    "zasr_fbank_set_mel_banks", "zasr_selftest_launch", "zasr_decode_host_batches",
    "zasr_selftest_gemm_h3r", "zasr_selftest_ffn_h3", "zasr_selftest_ffn_bf16",
)


# include/zasr.h ZASR_PRECISION_*: "bf16_enc" = the bf16 encoder with the f32 joiner + search;
# "bf16x3" / "bf16x6" = f32 storage, split-bf16 products (2 / 3 pieces per operand) on the
# bf16 MFMA
PRECISIONS = {"fp32": 0, "bf16": 1, "bf16_enc": 2, "bf16x3": 3, "bf16x6": 4, "f16x3": 5}


C_FP = C.POINTER(C.c_float)


class ZasrError(RuntimeError):
    pass


class _Config(C.Structure):
    _fields_ = [
        ("model_dir", C.c_char_p),
        ("decoding_method", C.c_char_p),
        ("max_active_paths", C.c_int32),
        ("blank_penalty", C.c_float),
        ("hotword_tokens", C.POINTER(C.c_int32)),
        ("hotword_lens", C.POINTER(C.c_int32)),
        ("hotword_scores", C.POINTER(C.c_float)),
        ("num_hotwords", C.c_int32),
        ("device_id", C.c_int32),
        ("precision", C.c_int32),
    ]


_lib = None


def load_library(path: Optional[str] = None) -> C.CDLL:
    """Load libzasr.so (raises if absent: the product has no fallback path)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("ZASR_LIB", DEFAULT_LIB)
    if not os.path.exists(p):
        raise ZasrError(f"libzasr.so not found at {p}; build it with "
                        f"`make -C sherpa-vietnamese-asr_amd/csrc` (or __graft_entry__.build())")
    lib = C.CDLL(p)
    P, I32, I64 = C.c_void_p, C.c_int32, C.c_int64
    fp = C.POINTER(C.c_float)
    lib.zasr_create.argtypes = [C.POINTER(_Config), C.POINTER(P)]
    lib.zasr_create.restype = C.c_int
    lib.zasr_destroy.argtypes = [P]
    lib.zasr_destroy.restype = None
    lib.zasr_convert_model.argtypes = [C.c_char_p, C.c_char_p]
    lib.zasr_convert_model.restype = C.c_int
    lib.zasr_convert_stage_model.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p]
    lib.zasr_convert_stage_model.restype = C.c_int
    lib.zasr_fbank.argtypes = [P, fp, I64, I32, fp, I64, C.POINTER(I64)]
    lib.zasr_fbank.restype = C.c_int
    lib.zasr_decode_batch.argtypes = [P, C.POINTER(fp), C.POINTER(I64), I32, I32, C.POINTER(P)]
    lib.zasr_decode_batch.restype = C.c_int
    lib.zasr_decode_features.argtypes = [P, C.POINTER(fp), C.POINTER(I64), I32, I32, C.POINTER(P)]
    lib.zasr_decode_features.restype = C.c_int
    lib.zasr_decode_device.argtypes = [P, P, C.POINTER(I64), C.POINTER(I64), I32, I32, P,
                                       C.POINTER(P)]
    lib.zasr_decode_device.restype = C.c_int
    lib.zasr_decode_device_batches.argtypes = [P, P, C.POINTER(I64), C.POINTER(I64), I32,
                                               C.POINTER(I32), I32, I32, P, C.POINTER(P)]
    lib.zasr_decode_device_batches.restype = C.c_int
    lib.zasr_decode_host_batches.argtypes = [P, P, C.POINTER(I64), C.POINTER(I64), I32,
                                             C.POINTER(I32), I32, I32, P, C.POINTER(P)]
    lib.zasr_decode_host_batches.restype = C.c_int
    lib.zasr_encode_features.argtypes = [P, C.POINTER(fp), C.POINTER(I64), I32, fp, I64,
                                         C.POINTER(I64)]
    lib.zasr_encode_features.restype = C.c_int
    lib.zasr_search_encoder_out.argtypes = [P, C.POINTER(fp), C.POINTER(I64), I32, I32,
                                            C.POINTER(P)]
    lib.zasr_search_encoder_out.restype = C.c_int
    for n in ("zasr_result_count",):
        getattr(lib, n).argtypes = [P]
        getattr(lib, n).restype = I32
    for n in ("zasr_result_num_tokens", "zasr_result_num_frames"):
        getattr(lib, n).argtypes = [P, I32]
        getattr(lib, n).restype = I32
    lib.zasr_result_tokens.argtypes = [P, I32]
    lib.zasr_result_tokens.restype = C.POINTER(I32)
    lib.zasr_result_frames.argtypes = [P, I32]
    lib.zasr_result_frames.restype = C.POINTER(I32)
    lib.zasr_result_log_probs.argtypes = [P, I32]
    lib.zasr_result_log_probs.restype = C.POINTER(C.c_double)
    lib.zasr_result_token_stats.argtypes = [P, I32]
    lib.zasr_result_token_stats.restype = fp
    lib.zasr_result_free.argtypes = [P]
    lib.zasr_result_free.restype = None
    lib.zasr_vocab_size.argtypes = [P]
    lib.zasr_vocab_size.restype = I32
    lib.zasr_joiner_dim.argtypes = [P]
    lib.zasr_joiner_dim.restype = I32
    lib.zasr_profile_enable.argtypes = [P, I32]
    lib.zasr_profile_enable.restype = C.c_int
    lib.zasr_profile_reset.argtypes = [P]
    lib.zasr_profile_reset.restype = C.c_int
    lib.zasr_profile_report.argtypes = [P, C.c_char_p, I64]
    lib.zasr_profile_report.restype = C.c_int
    lib.zasr_last_error.argtypes = []
    lib.zasr_last_error.restype = C.c_char_p
    lib.zasr_version.argtypes = []
    lib.zasr_version.restype = C.c_char_p
    lib.zasr_campp_create.argtypes = [C.c_char_p, I32, C.POINTER(P)]
    lib.zasr_campp_create.restype = C.c_int
    lib.zasr_campp_destroy.argtypes = [P]
    lib.zasr_campp_destroy.restype = None
    lib.zasr_campp_embedding_dim.argtypes = [P]
    lib.zasr_campp_embedding_dim.restype = I32
    lib.zasr_campp_fbank.argtypes = [P, fp, I64, fp, I64, C.POINTER(I64)]
    lib.zasr_campp_fbank.restype = C.c_int
    lib.zasr_campp_embed.argtypes = [P, fp, I32, I32, fp]
    lib.zasr_campp_embed.restype = C.c_int
    lib.zasr_campp_embed_device.argtypes = [P, P, I32, I32, P, P]
    lib.zasr_campp_embed_device.restype = C.c_int
    i32p = C.POINTER(I32)
    lib.zasr_campp_windows_device.argtypes = [P, P, C.POINTER(I64), C.POINTER(I64), I32, I32, I32,
                                              P, I64, i32p, i32p, i32p, C.POINTER(I64), P]
    lib.zasr_campp_windows_device.restype = C.c_int
    lib.zasr_vibert_create.argtypes = [C.c_char_p, I32, C.POINTER(P)]
    lib.zasr_vibert_create.restype = C.c_int
    lib.zasr_vibert_destroy.argtypes = [P]
    lib.zasr_vibert_destroy.restype = None
    for n in ("zasr_vibert_num_labels", "zasr_vibert_num_detect"):
        getattr(lib, n).argtypes = [P]
        getattr(lib, n).restype = I32
    i64p = C.POINTER(I64)
    lib.zasr_vibert_run.argtypes = [P, i64p, i64p, i64p, i64p, I32, I32, I32, fp, fp]
    lib.zasr_vibert_run.restype = C.c_int
    lib.zasr_vad_create.argtypes = [C.c_char_p, I32, C.POINTER(P)]
    lib.zasr_vad_create.restype = C.c_int
    lib.zasr_vad_destroy.argtypes = [P]
    lib.zasr_vad_destroy.restype = None
    lib.zasr_vad_probs.argtypes = [P, fp, i64p, i64p, I32, I32, fp]
    lib.zasr_vad_probs.restype = C.c_int
    lib.zasr_vad_probs_device.argtypes = [P, P, i64p, i64p, I32, I32, P, P]
    lib.zasr_vad_probs_device.restype = C.c_int
    lib.zasr_vad_window.argtypes = [P, fp, fp, I32, fp, fp]
    lib.zasr_vad_window.restype = C.c_int
    lib.zasr_vad_last_passes.argtypes = [P]
    lib.zasr_vad_last_passes.restype = I32
    lib.zasr_silence_flags.argtypes = [P, I64, I32, C.c_float, P, P]
    lib.zasr_silence_flags.restype = C.c_int
    # offline streams (the sherpa-onnx OfflineStream surface, zasr/offline.py)
    lib.zasr_create_stream.argtypes = [P, C.POINTER(P)]
    lib.zasr_create_stream.restype = C.c_int
    lib.zasr_destroy_stream.argtypes = [P]
    lib.zasr_destroy_stream.restype = None
    lib.zasr_stream_accept_waveform.argtypes = [P, I32, fp, I64]
    lib.zasr_stream_accept_waveform.restype = C.c_int
    lib.zasr_decode_stream.argtypes = [P, P]
    lib.zasr_decode_stream.restype = C.c_int
    lib.zasr_decode_streams.argtypes = [P, C.POINTER(P), I32]
    lib.zasr_decode_streams.restype = C.c_int
    for n in ("zasr_stream_is_decoded", "zasr_stream_num_tokens", "zasr_stream_num_frames"):
        getattr(lib, n).argtypes = [P]
        getattr(lib, n).restype = I32
    lib.zasr_stream_tokens.argtypes = [P]
    lib.zasr_stream_tokens.restype = C.POINTER(I32)
    lib.zasr_stream_frames.argtypes = [P]
    lib.zasr_stream_frames.restype = C.POINTER(I32)
    lib.zasr_stream_log_probs.argtypes = [P]
    lib.zasr_stream_log_probs.restype = C.POINTER(C.c_double)
    lib.zasr_stream_token_stats.argtypes = [P]
    lib.zasr_stream_token_stats.restype = fp
    lib.zasr_stream_result_json.argtypes = [P, C.c_char_p, I64, C.POINTER(I64)]
    lib.zasr_stream_result_json.restype = C.c_int
    lib.zasr_set_tokens.argtypes = [P, C.c_char_p]
    lib.zasr_set_tokens.restype = C.c_int
    lib.zasr_model_routes.argtypes = [P, C.c_char_p, I64]
    lib.zasr_model_routes.restype = C.c_int
    lib.zasr_fbank_set_mel_banks.argtypes = [P, fp, I32]
    lib.zasr_fbank_set_mel_banks.restype = C.c_int
    lib.zasr_selftest_launch.argtypes = [I32]
    lib.zasr_selftest_launch.restype = C.c_int
    lib.zasr_selftest_gemm_h3r.argtypes = [I32, I32, I32, I32, fp, fp, fp, fp]
    lib.zasr_selftest_gemm_h3r.restype = C.c_int
    lib.zasr_selftest_ffn_h3.argtypes = [I32, I32, I32, fp, fp, fp, fp, fp, fp, fp, fp]
    lib.zasr_selftest_ffn_h3.restype = C.c_int
    lib.zasr_selftest_ffn_bf16.argtypes = [I32, I32, I32, fp, fp, fp, fp, fp, fp, fp, I32]
    lib.zasr_selftest_ffn_bf16.restype = C.c_int
    if path is None:
        _lib = lib
    return lib


def convert_model(model_dir: str, out_dir: str, lib_path: Optional[str] = None) -> None:
    """Host-only load of a model directory (config.json + model.safetensors, or the
    reference's encoder-/decoder-/joiner-*.onnx) through libzasr's loader, written as
    out_dir/config.json + out_dir/model.safetensors (include/zasr.h zasr_convert_model)."""
    lib = load_library(lib_path)
    os.makedirs(out_dir, exist_ok=True)
    rc = lib.zasr_convert_model(model_dir.encode(), out_dir.encode())
    if rc != 0:
        msg = lib.zasr_last_error().decode()
        if rc == 2:
            raise FileNotFoundError(msg)
        raise ZasrError(msg)


def convert_stage_model(kind: str, model_dir: str, out_dir: str,
                        lib_path: Optional[str] = None) -> None:
    """Host-only load of a Silero VAD / CAM++ / ViBERT model directory (the reference's .onnx
    or the engine's own files) through libzasr's reader, written as out_dir/<kind>_config.json
    + the engine's safetensors file (include/zasr.h zasr_convert_stage_model)."""
    lib = load_library(lib_path)
    os.makedirs(out_dir, exist_ok=True)
    rc = lib.zasr_convert_stage_model(kind.encode(), model_dir.encode(), out_dir.encode())
    if rc != 0:
        msg = lib.zasr_last_error().decode()
        if rc == 2:
            raise FileNotFoundError(msg)
        raise ZasrError(msg)


def selftest_launch(block_threads: int, lib_path: Optional[str] = None) -> None:
    """A no-op kernel of block_threads threads through the library's checked launch path
    (include/zasr.h zasr_selftest_launch): an invalid configuration raises ZasrError."""
    lib = load_library(lib_path)
    rc = lib.zasr_selftest_launch(int(block_threads))
    if rc != 0:
        raise ZasrError(lib.zasr_last_error().decode())


def selftest_gemm_h3r(A, W, bias, C, epi: int = 0, lib_path: Optional[str] = None) -> np.ndarray:
    """gemm_h3r_kernel alone on host operands (zasr_selftest_gemm_h3r): returns C after
    C = epi(A W^T + bias) (epi 3: C += ..., 8: GLU over interleaved rows)."""
    lib = load_library(lib_path)
    A, W, C = _f32(A), _f32(W), _f32(C).copy()
    b = None if bias is None else _f32(bias)
    p = lambda x: None if x is None else x.ctypes.data_as(C_FP)
    rc = lib.zasr_selftest_gemm_h3r(A.shape[0], A.shape[1], W.shape[0], int(epi), p(A), p(W),
                                    p(b), p(C))
    if rc != 0:
        raise ZasrError(lib.zasr_last_error().decode())
    return C


def selftest_ffn_h3(Y, W1, b1, W2, b2, X, byp_orig=None, byp_scale=None,
                    lib_path: Optional[str] = None) -> np.ndarray:
    """ffn_wide_h3_kernel alone on host operands (zasr_selftest_ffn_h3): returns
    X + W2 SwooshL(W1 Y + b1) + b2 (then the bypass_mid blend when byp_orig is given)."""
    lib = load_library(lib_path)
    Y, W1, b1, W2, b2, X = (_f32(v) for v in (Y, W1, b1, W2, b2, X))
    X = X.copy()
    bo = None if byp_orig is None else _f32(byp_orig)
    bs = None if byp_scale is None else _f32(byp_scale)
    p = lambda x: None if x is None else x.ctypes.data_as(C_FP)
    rc = lib.zasr_selftest_ffn_h3(Y.shape[0], Y.shape[1], W1.shape[0], p(Y), p(W1), p(b1), p(W2),
                                  p(b2), p(bo), p(bs), p(X))
    if rc != 0:
        raise ZasrError(lib.zasr_last_error().decode())
    return X


def selftest_ffn_bf16(W1, b1, W2, b2, X, byp_orig=None, byp_scale=None, form: int = 0,
                      lib_path: Optional[str] = None) -> np.ndarray:
    """The bf16 fused FFN alone on host operands (zasr_selftest_ffn_bf16): returns
    X + W2 SwooshL(W1 bf16(X) + b1) + b2 (bf16 weights and hidden activation; then the
    bypass_mid blend when byp_orig is given).  form 1: the opt-in rows form at D = 384."""
    lib = load_library(lib_path)
    W1, b1, W2, b2, X = (_f32(v) for v in (W1, b1, W2, b2, X))
    X = X.copy()
    bo = None if byp_orig is None else _f32(byp_orig)
    bs = None if byp_scale is None else _f32(byp_scale)
    p = lambda x: None if x is None else x.ctypes.data_as(C_FP)
    rc = lib.zasr_selftest_ffn_bf16(X.shape[0], X.shape[1], W1.shape[0], p(W1), p(b1), p(W2),
                                    p(b2), p(bo), p(bs), p(X), int(form))
    if rc != 0:
        raise ZasrError(lib.zasr_last_error().decode())
    return X


def silence_flags(d_wav_ptr: int, n: int, frame_len: int, threshold: float, d_flags_ptr: int,
                  stream: int = 0, lib_path: Optional[str] = None) -> None:
    """Per-frame silence flags of an HBM-resident signal (include/zasr.h zasr_silence_flags):
    d_flags[f] = sqrt(mean(frame_f ** 2)) < threshold in numpy float32 arithmetic."""
    lib = load_library(lib_path)
    rc = lib.zasr_silence_flags(C.c_void_p(d_wav_ptr), int(n), int(frame_len),
                                float(threshold), C.c_void_p(d_flags_ptr), C.c_void_p(stream))
    if rc != 0:
        raise ZasrError(lib.zasr_last_error().decode())


@dataclasses.dataclass
class SearchResult:
    """One chunk's search output: the tuple of core/asr_engine.py:1153 with per-token
    entropy statistics (entropy, sum p^(1/3), top1, top2) in place of raw logits rows."""
    token_ids: np.ndarray
    frames: np.ndarray
    log_probs: np.ndarray
    stats: np.ndarray
    T: int


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _ptr_array(arrs: Sequence[np.ndarray]):
    fp = C.POINTER(C.c_float)
    return (fp * len(arrs))(*[a.ctypes.data_as(fp) for a in arrs])


class Recognizer:
    def __init__(self, model_dir: str, decoding_method: str = "modified_beam_search",
                 max_active_paths: int = 8, hotwords: Optional[Sequence[Sequence[int]]] = None,
                 hotword_scores: Optional[Sequence[float]] = None, device_id: int = 0,
                 precision: str = "fp32", lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        hotwords = [list(map(int, h)) for h in (hotwords or [])]
        scores = list(hotword_scores or [1.5] * len(hotwords))
        flat = np.array([t for h in hotwords for t in h] or [0], dtype=np.int32)
        lens = np.array([len(h) for h in hotwords] or [0], dtype=np.int32)
        sc = np.array(scores or [0.0], dtype=np.float32)
        self._keep = (flat, lens, sc)
        cfg = _Config(model_dir.encode(), decoding_method.encode(), max_active_paths, 0.0,
                      flat.ctypes.data_as(C.POINTER(C.c_int32)),
                      lens.ctypes.data_as(C.POINTER(C.c_int32)),
                      sc.ctypes.data_as(C.POINTER(C.c_float)), len(hotwords), device_id,
                      PRECISIONS[precision])
        h = C.c_void_p()
        rc = self.lib.zasr_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            msg = self.lib.zasr_last_error().decode()
            if rc == 2:
                raise FileNotFoundError(msg)
            raise ZasrError(msg)
        self.handle = h
        self.device_id = int(device_id)
        self.precision = precision
        self.vocab_size = self.lib.zasr_vocab_size(h)
        self.joiner_dim = self.lib.zasr_joiner_dim(h)
        self._args = (model_dir, decoding_method, max_active_paths, hotwords, scores, device_id,
                      lib_path)
        self._fallback = None

    def close(self):
        if getattr(self, "handle", None):
            self.lib.zasr_destroy(self.handle)
            self.handle = None
        fb = getattr(self, "_fallback", None)
        if fb is not None:
            fb.close()
            self._fallback = None

    # f16x3 stores the split operands as fp16 pieces (|x| < 65504); an activation beyond that
    # range makes the encoder output non-finite, which the engine detects per batch (after
    # draining every stream) and reports.  The decode is then redone by a bf16x6 engine of the
    # same model: the other exact-f32-quality mode, whose bf16 pieces have f32's range
    # (DESIGN.md §6), so the caller still gets the token-exact transcript.
    FALLBACK_PRECISION = "bf16x6"

    def _retry(self, e: "ZasrError", name: str, *args, **kw):
        if self.precision != "f16x3" or "non-finite encoder output" not in str(e):
            raise e
        if self._fallback is None:
            import logging
            logging.getLogger("zasr").warning(
                "[zasr] f16x3 operand range exceeded; re-decoding with %s", self.FALLBACK_PRECISION)
            md, method, beam, hw, sc, dev, lp = self._args
            self._fallback = Recognizer(md, method, beam, hotwords=hw, hotword_scores=sc,
                                        device_id=dev, precision=self.FALLBACK_PRECISION,
                                        lib_path=lp)
        return getattr(self._fallback, name)(*args, **kw)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise ZasrError(self.lib.zasr_last_error().decode())

    def _collect(self, res) -> List[SearchResult]:
        out = []
        try:
            n = self.lib.zasr_result_count(res)
            for i in range(n):
                k = self.lib.zasr_result_num_tokens(res, i)
                T = self.lib.zasr_result_num_frames(res, i)
                if k > 0:
                    tok = np.ctypeslib.as_array(self.lib.zasr_result_tokens(res, i), (k,)).copy()
                    fr = np.ctypeslib.as_array(self.lib.zasr_result_frames(res, i), (k,)).copy()
                    lp = np.ctypeslib.as_array(self.lib.zasr_result_log_probs(res, i), (k,)).copy()
                    st = np.ctypeslib.as_array(self.lib.zasr_result_token_stats(res, i),
                                               (k * 4,)).copy().reshape(k, 4)
                else:
                    tok = np.zeros(0, np.int32)
                    fr = np.zeros(0, np.int32)
                    lp = np.zeros(0, np.float64)
                    st = np.zeros((0, 4), np.float32)
                out.append(SearchResult(tok, fr, lp, st, T))
        finally:
            self.lib.zasr_result_free(res)
        return out

    def routes(self) -> dict:
        """Which kernel each part of the loaded model was routed to (zasr_model_routes)."""
        import json
        buf = C.create_string_buffer(1024)
        self._check(self.lib.zasr_model_routes(self.handle, buf, len(buf)))
        return json.loads(buf.value.decode())

    def set_mel_banks(self, banks) -> None:
        """Replace the fbank's 80 triangular filters ([80][256] or [80][257] weights;
        zasr_fbank_set_mel_banks)."""
        b = _f32(banks)
        if b.ndim != 2 or b.shape[0] != 80 or b.shape[1] not in (256, 257):
            raise ValueError("mel banks must be [80][256] or [80][257]")
        self._check(self.lib.zasr_fbank_set_mel_banks(
            self.handle, b.ctypes.data_as(C.POINTER(C.c_float)), b.shape[1]))

    def fbank(self, audio) -> np.ndarray:
        a = _f32(audio)
        n = a.shape[0]
        frames = (n + 80) // 160 if n > 0 else 0
        out = np.empty((max(frames, 1), 80), dtype=np.float32)
        nf = C.c_int64()
        fp = C.POINTER(C.c_float)
        self._check(self.lib.zasr_fbank(self.handle, a.ctypes.data_as(fp), n, 16000,
                                        out.ctypes.data_as(fp), out.size, C.byref(nf)))
        return out[: nf.value]

    def decode(self, chunks: Sequence, beam: int = 0) -> List[SearchResult]:
        arrs = [_f32(c) for c in chunks]
        ns = (C.c_int64 * len(arrs))(*[a.shape[0] for a in arrs])
        res = C.c_void_p()
        try:
            self._check(self.lib.zasr_decode_batch(self.handle, _ptr_array(arrs), ns, len(arrs),
                                                   beam, C.byref(res)))
        except ZasrError as e:
            return self._retry(e, "decode", arrs, beam=beam)
        return self._collect(res)

    def decode_features(self, feats: Sequence, beam: int = 0) -> List[SearchResult]:
        arrs = [_f32(f) for f in feats]
        ns = (C.c_int64 * len(arrs))(*[a.shape[0] for a in arrs])
        res = C.c_void_p()
        try:
            self._check(self.lib.zasr_decode_features(self.handle, _ptr_array(arrs), ns,
                                                      len(arrs), beam, C.byref(res)))
        except ZasrError as e:
            return self._retry(e, "decode_features", arrs, beam=beam)
        return self._collect(res)

    def decode_device(self, d_wav_ptr: int, offsets: Sequence[int], lengths: Sequence[int],
                      beam: int = 0, stream: int = 0) -> List[SearchResult]:
        n = len(lengths)
        off = (C.c_int64 * n)(*offsets)
        ln = (C.c_int64 * n)(*lengths)
        res = C.c_void_p()
        try:
            self._check(self.lib.zasr_decode_device(self.handle, C.c_void_p(d_wav_ptr), off, ln,
                                                    n, beam, C.c_void_p(stream), C.byref(res)))
        except ZasrError as e:
            return self._retry(e, "decode_device", d_wav_ptr, offsets, lengths, beam=beam,
                               stream=stream)
        return self._collect(res)

    def decode_device_batches(self, d_wav_ptr: int, offsets: Sequence[int],
                              lengths: Sequence[int], batch_sizes: Sequence[int],
                              beam: int = 0, stream: int = 0) -> List[SearchResult]:
        """Consecutive batches (batch_sizes[i] chunks each) decoded with batch k+1's encoder
        overlapping batch k's search; results for every chunk, in chunk order."""
        n = len(lengths)
        off = (C.c_int64 * n)(*offsets)
        ln = (C.c_int64 * n)(*lengths)
        bs = (C.c_int32 * len(batch_sizes))(*batch_sizes)
        res = C.c_void_p()
        try:
            self._check(self.lib.zasr_decode_device_batches(
                self.handle, C.c_void_p(d_wav_ptr), off, ln, n, bs, len(batch_sizes), beam,
                C.c_void_p(stream), C.byref(res)))
        except ZasrError as e:
            return self._retry(e, "decode_device_batches", d_wav_ptr, offsets, lengths,
                               batch_sizes, beam=beam, stream=stream)
        return self._collect(res)

    def decode_host_batches(self, h_wav_ptr: int, offsets: Sequence[int],
                            lengths: Sequence[int], batch_sizes: Sequence[int],
                            beam: int = 0, stream: int = 0) -> List[SearchResult]:
        """decode_device_batches from HOST waveforms at h_wav_ptr (pinned for an asynchronous
        upload): each batch's samples are copied on the engine's copy stream under the
        previous batch's work (zasr_decode_host_batches)."""
        n = len(lengths)
        off = (C.c_int64 * n)(*offsets)
        ln = (C.c_int64 * n)(*lengths)
        bs = (C.c_int32 * len(batch_sizes))(*batch_sizes)
        res = C.c_void_p()
        try:
            self._check(self.lib.zasr_decode_host_batches(
                self.handle, C.c_void_p(h_wav_ptr), off, ln, n, bs, len(batch_sizes), beam,
                C.c_void_p(stream), C.byref(res)))
        except ZasrError as e:
            return self._retry(e, "decode_host_batches", h_wav_ptr, offsets, lengths,
                               batch_sizes, beam=beam, stream=stream)
        return self._collect(res)

    def encode_features(self, feats: Sequence) -> List[np.ndarray]:
        arrs = [_f32(f) for f in feats]
        ns = (C.c_int64 * len(arrs))(*[a.shape[0] for a in arrs])
        tot = sum(((a.shape[0] - 7) // 2 + 1) // 2 for a in arrs)
        out = np.empty((max(tot, 1), self.joiner_dim), dtype=np.float32)
        tout = (C.c_int64 * len(arrs))()
        fp = C.POINTER(C.c_float)
        self._check(self.lib.zasr_encode_features(self.handle, _ptr_array(arrs), ns, len(arrs),
                                                  out.ctypes.data_as(fp), out.size, tout))
        res, pos = [], 0
        for i in range(len(arrs)):
            res.append(out[pos: pos + tout[i]].copy())
            pos += tout[i]
        return res

    def search(self, enc_outs: Sequence, beam: int = 0) -> List[SearchResult]:
        arrs = [_f32(e).reshape(-1, self.joiner_dim) for e in enc_outs]
        ns = (C.c_int64 * len(arrs))(*[a.shape[0] for a in arrs])
        res = C.c_void_p()
        self._check(self.lib.zasr_search_encoder_out(self.handle, _ptr_array(arrs), ns,
                                                     len(arrs), beam, C.byref(res)))
        return self._collect(res)

    # profiling (HIP events on the library's stream)
    def profile(self, on=True):
        """on: False/0 off, True/1 kernel classes, 2 = GEMMs split by shape."""
        self._check(self.lib.zasr_profile_enable(self.handle, int(on)))

    def profile_reset(self):
        self._check(self.lib.zasr_profile_reset(self.handle))

    def profile_report(self) -> dict:
        buf = C.create_string_buffer(1 << 16)
        self._check(self.lib.zasr_profile_report(self.handle, buf, len(buf)))
        out = {}
        for line in buf.value.decode().splitlines():
            name, cnt, ms = line.split()
            out[name] = (int(cnt), float(ms))
        return out


class CamppEmbedder:
    """CAM++ speaker embeddings on the GPU (include/zasr.h zasr_campp_*): the reference's
    numpy fbank (core/speaker_diarization_senko_campp_optimized.py:86-159) and its batched
    ONNX CAM++ session (:589-605)."""

    def __init__(self, model_dir: str, device_id: int = 0, lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        rc = self.lib.zasr_campp_create(model_dir.encode(), device_id, C.byref(h))
        if rc != 0:
            msg = self.lib.zasr_last_error().decode()
            if rc == 2:
                raise FileNotFoundError(msg)
            raise ZasrError(msg)
        self.handle = h
        self.dim = self.lib.zasr_campp_embedding_dim(h)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.zasr_campp_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise ZasrError(self.lib.zasr_last_error().decode())

    def routes(self) -> dict:
        """Which kernel each part of the loaded model was routed to (zasr_model_routes)."""
        import json
        buf = C.create_string_buffer(1024)
        self._check(self.lib.zasr_model_routes(self.handle, buf, len(buf)))
        return json.loads(buf.value.decode())

    def set_mel_banks(self, banks) -> None:
        """Replace the fbank's 80 triangular filters ([80][256] or [80][257] weights;
        zasr_fbank_set_mel_banks)."""
        b = _f32(banks)
        if b.ndim != 2 or b.shape[0] != 80 or b.shape[1] not in (256, 257):
            raise ValueError("mel banks must be [80][256] or [80][257]")
        self._check(self.lib.zasr_fbank_set_mel_banks(
            self.handle, b.ctypes.data_as(C.POINTER(C.c_float)), b.shape[1]))

    def fbank(self, audio) -> np.ndarray:
        a = _f32(audio)
        n = a.shape[0]
        frames = 1 + (n - 400) // 160 if n >= 400 else 0
        out = np.empty((max(frames, 1), 80), dtype=np.float32)
        nf = C.c_int64()
        fp = C.POINTER(C.c_float)
        self._check(self.lib.zasr_campp_fbank(self.handle, a.ctypes.data_as(fp), n,
                                              out.ctypes.data_as(fp), out.size, C.byref(nf)))
        return out[: nf.value]

    def embed(self, feats) -> np.ndarray:
        x = _f32(feats)
        if x.ndim != 3 or x.shape[2] != 80:
            raise ValueError("feats must be [N, T, 80]")
        out = np.empty((x.shape[0], self.dim), dtype=np.float32)
        fp = C.POINTER(C.c_float)
        self._check(self.lib.zasr_campp_embed(self.handle, x.ctypes.data_as(fp), x.shape[0],
                                              x.shape[1], out.ctypes.data_as(fp)))
        return out

    def embed_device(self, d_feats: int, count: int, n_frames: int, d_out: int, stream: int = 0):
        self._check(self.lib.zasr_campp_embed_device(self.handle, C.c_void_p(d_feats), count,
                                                     n_frames, C.c_void_p(d_out),
                                                     C.c_void_p(stream)))


    def windows_device(self, d_wav: int, region_off: Sequence[int], region_len: Sequence[int],
                       d_feats: int, max_windows: int, window_frames: int = 150,
                       step_frames: int = 60, stream: int = 0):
        """fbank + CMVN of every speech region of a waveform in HBM and its 1.5 s windows
        gathered into d_feats [n][window_frames][80] (zasr_campp_windows_device; the reference's
        _sliding_window_embeddings front end, core/speaker_diarization_senko_campp_optimized.py:
        540-600).  Returns (region, first frame, frame count) int32 arrays of the n windows."""
        off = np.ascontiguousarray(region_off, dtype=np.int64)
        ln = np.ascontiguousarray(region_len, dtype=np.int64)
        if off.shape != ln.shape:
            raise ValueError("region_off and region_len differ in length")
        cap = max(0, int(max_windows))
        reg = np.empty(max(cap, 1), np.int32)
        first = np.empty(max(cap, 1), np.int32)
        nfr = np.empty(max(cap, 1), np.int32)
        n = C.c_int64()
        i64p = C.POINTER(C.c_int64)
        i32p = C.POINTER(C.c_int32)
        self._check(self.lib.zasr_campp_windows_device(
            self.handle, C.c_void_p(d_wav), off.ctypes.data_as(i64p), ln.ctypes.data_as(i64p),
            off.size, window_frames, step_frames, C.c_void_p(d_feats), cap,
            reg.ctypes.data_as(i32p), first.ctypes.data_as(i32p), nfr.ctypes.data_as(i32p),
            C.byref(n), C.c_void_p(stream)))
        k = n.value
        return reg[:k], first[:k], nfr[:k]


class VibertSession:
    """ViBERT-capu on the GPU with the onnxruntime InferenceSession surface the reference's
    GecBERTModel uses (core/gec_model.py:366-412): run(None, feeds) -> [logits,
    detect_logits] for feeds {input_ids, attention_mask, token_type_ids, input_offsets}."""

    def __init__(self, model_dir: str, device_id: int = 0, lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        rc = self.lib.zasr_vibert_create(model_dir.encode(), device_id, C.byref(h))
        if rc != 0:
            msg = self.lib.zasr_last_error().decode()
            if rc == 2:
                raise FileNotFoundError(msg)
            raise ZasrError(msg)
        self.handle = h
        self.num_labels = self.lib.zasr_vibert_num_labels(h)
        self.num_detect = self.lib.zasr_vibert_num_detect(h)

    def close(self):
        if getattr(self, "handle", None):
            self.lib.zasr_vibert_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, output_names, feeds):
        i64 = lambda k: np.ascontiguousarray(np.asarray(feeds[k]), dtype=np.int64)  # noqa: E731
        ids, am, tt, off = (i64(k) for k in ("input_ids", "attention_mask", "token_type_ids",
                                              "input_offsets"))
        B, L = ids.shape
        W = off.shape[1]
        lg = np.empty((B, W, self.num_labels), np.float32)
        dl = np.empty((B, W, self.num_detect), np.float32)
        p = lambda a: a.ctypes.data_as(C.POINTER(C.c_int64))  # noqa: E731
        fp = C.POINTER(C.c_float)
        rc = self.lib.zasr_vibert_run(self.handle, p(ids), p(am), p(tt), p(off), B, L, W,
                                      lg.ctypes.data_as(fp), dl.ctypes.data_as(fp))
        if rc != 0:
            raise ZasrError(self.lib.zasr_last_error().decode())
        outs = {"logits": lg, "detect_logits": dl}
        return [lg, dl] if output_names is None else [outs[n] for n in output_names]


class VadSession:
    """Silero VAD on the GPU.  probs() runs whole files (the reference's
    per-window loop at core/vad_utils.py:80-111, batched); run(None, feeds) is the
    onnxruntime session surface ({input [n, 576], state [2, n, 128], sr} -> [prob [n, 1],
    state]) for the reference's per-window callers."""

    def __init__(self, model_dir: str, device_id: int = 0, lib_path: Optional[str] = None):
        self.lib = load_library(lib_path)
        h = C.c_void_p()
        rc = self.lib.zasr_vad_create(model_dir.encode(), device_id, C.byref(h))
        if rc != 0:
            msg = self.lib.zasr_last_error().decode()
            if rc == 2:
                raise FileNotFoundError(msg)
            raise ZasrError(msg)
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self.lib.zasr_vad_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise ZasrError(self.lib.zasr_last_error().decode())

    def probs(self, audios: Sequence[np.ndarray], auto_boost: bool = False) -> List[np.ndarray]:
        audios = [np.ascontiguousarray(a, np.float32) for a in audios]
        lens = np.array([a.shape[0] for a in audios], np.int64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        flat = np.concatenate(audios) if audios else np.zeros(0, np.float32)
        nw = lens // 512
        out = np.empty(int(nw.sum()), np.float32)
        fp = C.POINTER(C.c_float)
        i64 = C.POINTER(C.c_int64)
        if out.size:
            self._check(self.lib.zasr_vad_probs(self.handle, flat.ctypes.data_as(fp),
                                                offs.ctypes.data_as(i64), lens.ctypes.data_as(i64),
                                                len(audios), int(auto_boost),
                                                out.ctypes.data_as(fp)))
        bounds = np.concatenate([[0], np.cumsum(nw)])
        return [out[bounds[i]:bounds[i + 1]] for i in range(len(audios))]

    @property
    def last_passes(self) -> int:
        return int(self.lib.zasr_vad_last_passes(self.handle))

    def probs_device(self, d_audio: int, offsets: Sequence[int], lengths: Sequence[int],
                     d_probs: int, auto_boost: bool = False, stream: int = 0) -> None:
        offs = np.ascontiguousarray(offsets, np.int64)
        lens = np.ascontiguousarray(lengths, np.int64)
        i64 = C.POINTER(C.c_int64)
        self._check(self.lib.zasr_vad_probs_device(
            self.handle, C.c_void_p(d_audio), offs.ctypes.data_as(i64), lens.ctypes.data_as(i64),
            len(offs), int(auto_boost), C.c_void_p(d_probs), C.c_void_p(stream)))

    def run(self, output_names, feeds):
        x = np.ascontiguousarray(feeds["input"], np.float32)
        st = np.ascontiguousarray(feeds["state"], np.float32)
        sr = int(np.asarray(feeds.get("sr", 16000)))
        if sr != 16000 or x.ndim != 2 or x.shape[1] != 576 or st.shape != (2, x.shape[0], 128):
            raise ZasrError("Silero VAD session: input [n, 576] at 16 kHz, state [2, n, 128]")
        n = x.shape[0]
        p = np.empty(n, np.float32)
        so = np.empty_like(st)
        fp = C.POINTER(C.c_float)
        self._check(self.lib.zasr_vad_window(self.handle, x.ctypes.data_as(fp),
                                             st.ctypes.data_as(fp), n, p.ctypes.data_as(fp),
                                             so.ctypes.data_as(fp)))
        return [p[:, None], so]
