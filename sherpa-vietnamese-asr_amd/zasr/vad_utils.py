"""Silero VAD on MI355X behind the reference's core/vad_utils.py interface.

  _get_vad_session      :17-38    -> VadSession: the ORT session surface (run(None, {input,
                                     state, sr})) on the GPU, for the per-window callers
                                     (streaming_asr.py:47-54, core/audio_analyzer.py:147-148)
  unload_vad_model      :41-48
  get_cached_vad_probs  :51-55
  _run_vad_inference    :62-151   all windows of the file in one GPU call (STFT, encoder and
                                  LSTM input projection batched over windows; the recurrence
                                  one workgroup per file), then the same segmentation
  get_vad_segments      :158-260  boost, retry at 0.3, fallback, padding, merge
  get_vad_segments_batch          MI355X-native: many files' VAD in one call (one LSTM
                                  workgroup per file), same per-file results

Model files: the reference's own models/silero-vad/silero_vad_16k_op15.onnx (or
silero_vad.onnx; read by libzasr's ONNX reader, onnx_io.cpp load_stage_onnx: the 16 kHz
branch's tensors found by walking the graph, LSTM gates reordered) or silero_config.json +
silero_vad.safetensors (zasr/silero.py), in $ZASR_VAD_MODEL_DIR, else <BASE_DIR>/models/
silero-vad of the installed reference.  A directory with neither raises FileNotFoundError,
which the reference's pipeline handles by falling back to silence chunking
(core/asr_engine.py:2171-2204).
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

WINDOW = 512
CONTEXT = 64
BOOST_TARGET = 0.071

_vad_session = None
_last_vad_probs: Optional[np.ndarray] = None
_lock = threading.Lock()
_BASE_DIR: Optional[str] = None   # set by zasr.dropin.install(..., vad_module=core.vad_utils)


def set_base_dir(base_dir: Optional[str]) -> None:
    global _BASE_DIR
    _BASE_DIR = base_dir


def model_dir() -> str:
    d = os.environ.get("ZASR_VAD_MODEL_DIR")
    if d:
        return d
    if _BASE_DIR is None:
        raise FileNotFoundError("Silero VAD model directory unknown: set ZASR_VAD_MODEL_DIR or "
                                "install() with the reference's core.vad_utils")
    return os.path.join(_BASE_DIR, "models", "silero-vad")


def _get_vad_session():
    """Lazily created GPU VAD engine (reference :17-38)."""
    global _vad_session
    with _lock:
        if _vad_session is None:
            from zasr.binding import VadSession
            d = model_dir()
            names = ("silero_config.json", "silero_vad_16k_op15.onnx", "silero_vad.onnx")
            if not any(os.path.isfile(os.path.join(d, n)) for n in names):
                raise FileNotFoundError(f"Silero VAD model (silero_vad_16k_op15.onnx, silero_vad.onnx "
                                        f"or silero_config.json + silero_vad.safetensors) not found in {d}")
            _vad_session = VadSession(d)
        return _vad_session


def unload_vad_model():
    global _vad_session, _last_vad_probs
    with _lock:
        if _vad_session is not None:
            _vad_session.close()
            _vad_session = None
    _last_vad_probs = None


def get_cached_vad_probs():
    return _last_vad_probs


def speech_windows(probs, threshold: float, min_silence_ms: int, min_speech_ms: int,
                   sample_rate: int = 16000) -> List[Tuple[int, int]]:
    """The reference's window state machine (:120-151), vectorized: runs of windows with
    prob >= threshold (compared in f64 like the reference's Python floats) joined across gaps
    shorter than the minimum silence; the last segment runs to the end unless a full minimum
    silence follows it; segments shorter than the minimum speech are dropped."""
    p = np.asarray(probs, np.float64)
    n = p.shape[0]
    if n == 0:
        return []
    min_sil = max(1, int(min_silence_ms * sample_rate / 1000 / WINDOW))
    min_sp = int(min_speech_ms * sample_rate / 1000 / WINDOW)
    a = np.concatenate([[0], (p >= threshold).astype(np.int8), [0]])
    d = np.diff(a)
    starts = np.flatnonzero(d == 1)
    ends = np.flatnonzero(d == -1)
    if starts.size == 0:
        return []
    brk = np.flatnonzero(starts[1:] - ends[:-1] >= min_sil)
    g_start = starts[np.concatenate([[0], brk + 1])]
    g_end = ends[np.concatenate([brk, [ends.size - 1]])].copy()
    if n - g_end[-1] < min_sil:
        g_end[-1] = n
    keep = g_end - g_start >= min_sp
    return [(int(s), int(e)) for s, e in zip(g_start[keep], g_end[keep])]


def _probs(audios: Sequence[np.ndarray], auto_boost: bool) -> List[np.ndarray]:
    return _get_vad_session().probs(audios, auto_boost=auto_boost)


def _run_vad_inference(audio, sample_rate=16000, threshold=0.5, min_silence_ms=300,
                       min_speech_ms=250, progress_callback=None):
    """Window-index speech segments of one file (reference :62-151)."""
    global _last_vad_probs
    audio = np.ascontiguousarray(audio, np.float32)
    if len(audio) // WINDOW == 0:
        return []
    probs = _probs([audio], False)[0]
    if progress_callback:
        progress_callback("PHASE:VAD|Đang phân tích audio|100")
    _last_vad_probs = probs
    return speech_windows(probs, threshold, min_silence_ms, min_speech_ms, sample_rate)


def _segments_from_probs(probs, total, sample_rate, threshold, min_silence_ms, min_speech_ms,
                         padding_ms, merge_gap_ms, fallback_full):
    segs = speech_windows(probs, threshold, min_silence_ms, min_speech_ms, sample_rate)
    if not segs:  # retry (:219-226): same probabilities, threshold 0.3, 100 / 150 ms
        segs = speech_windows(probs, 0.3, 100, 150, sample_rate)
    if not segs:
        return [(0, total)] if fallback_full else []
    pad = int(padding_ms * sample_rate / 1000)
    res = [(max(0, s * WINDOW - pad), min(total, e * WINDOW + pad)) for s, e in segs]
    if merge_gap_ms > 0 and len(res) > 1:
        gap = int(merge_gap_ms * sample_rate / 1000)
        merged = [res[0]]
        for s, e in res[1:]:
            if s - merged[-1][1] < gap:
                merged[-1] = (merged[-1][0], e)
            else:
                merged.append((s, e))
        res = merged
    return res


def get_vad_segments(audio, sample_rate=16000, threshold=0.2, min_silence_ms=100,
                     min_speech_ms=250, padding_ms=1000, merge_gap_ms=250, auto_boost=True,
                     fallback_full=True, progress_callback=None):
    """[(start_sample, end_sample)] speech segments of the original audio (reference
    :158-260)."""
    return get_vad_segments_batch([audio], sample_rate, threshold, min_silence_ms,
                                  min_speech_ms, padding_ms, merge_gap_ms, auto_boost,
                                  fallback_full, progress_callback)[0]


def get_vad_segments_batch(audios: Sequence[np.ndarray], sample_rate=16000, threshold=0.2,
                           min_silence_ms=100, min_speech_ms=250, padding_ms=1000,
                           merge_gap_ms=250, auto_boost=True, fallback_full=True,
                           progress_callback=None) -> List[List[Tuple[int, int]]]:
    """get_vad_segments for many files with one GPU call; per file the same result.
    get_cached_vad_probs() afterwards holds the last file's probabilities."""
    global _last_vad_probs
    if sample_rate != 16000:
        raise ValueError("Silero VAD runs at 16 kHz")
    audios = [np.ascontiguousarray(a, np.float32) for a in audios]
    out: List[Optional[List[Tuple[int, int]]]] = [None] * len(audios)
    todo = []
    for i, a in enumerate(audios):
        if len(a) < WINDOW:
            out[i] = [(0, len(a))] if fallback_full else []
        else:
            todo.append(i)
    if todo:
        probs = _probs([audios[i] for i in todo], auto_boost)
        if progress_callback:
            progress_callback("PHASE:VAD|Đang phân tích audio|100")
        for i, p in zip(todo, probs):
            out[i] = _segments_from_probs(p, len(audios[i]), sample_rate, threshold,
                                          min_silence_ms, min_speech_ms, padding_ms,
                                          merge_gap_ms, fallback_full)
        _last_vad_probs = probs[-1]
    return out  # type: ignore[return-value]
