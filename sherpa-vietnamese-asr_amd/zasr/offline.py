"""The sherpa-onnx OfflineRecognizer / OfflineStream surface over libzasr's stream C ABI.

The reference's callers outside the decode_chunk path bind sherpa-onnx's stream-shaped API:

  streaming_asr.py:224-243           sherpa_onnx.OfflineRecognizer.from_transducer(**kwargs)
                                     with tokens / encoder / decoder / joiner / num_threads /
                                     sample_rate / feature_dim / decoding_method /
                                     max_active_paths (+ hotwords_file / hotwords_score from
                                     core/config.py get_hotwords_config)
  core/audio_analyzer.py:345-361     stream = recognizer.create_stream();
                                     stream.accept_waveform(SAMPLE_RATE, audio);
                                     recognizer.decode_stream(stream); stream.result.text /
                                     .ys_log_probs
  sherpa-onnx-asr.js:1782-1880       the same through SherpaOnnxCreateOfflineStream /
                                     AcceptWaveformOffline / DecodeOfflineStream /
                                     GetOfflineStreamResultAsJson

`OfflineRecognizer` here has that surface; each call goes to the C ABI of include/zasr.h
(zasr_create_stream, zasr_stream_accept_waveform, zasr_decode_stream(s),
zasr_stream_result_json), so decode_streams([...]) is ONE batched GPU pass.  The result's
tokens, timestamps and ys_log_probs are those of the device search -- the same token ids and
log-probs decode_chunk's word dicts are built from (core/asr_engine.py:1209-1326).

Model files: the directory of `encoder` is loaded the way create_recognizer loads a model
directory (the reference's encoder-/decoder-/joiner-*.onnx set, non-int8 preferred, or this
build's config.json + model.safetensors); `tokens` is the symbol table (sherpa-onnx's
SymbolTable: a leading U+2581 is shown as a space, so `text` is the concatenation of the
token strings).  Hotword phrases are tokenized with the directory's bpe.model, as
create_recognizer does (no bpe.model: no hotwords).  16 kHz input only (the reference
resamples on load).  Precision: `precision=` or ZASR_PRECISION, default
zasr.asr_engine.DEFAULT_PRECISION.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import weakref
from typing import List, Optional, Sequence

import numpy as np

from zasr.binding import Recognizer, ZasrError


class OfflineRecognitionResult:
    """sherpa-onnx's OfflineRecognitionResult fields the reference reads (text, tokens,
    timestamps, ys_log_probs), plus the token ids, encoder frames and T'."""

    __slots__ = ("text", "tokens", "timestamps", "ys_log_probs", "token_ids", "frames",
                 "num_frames", "lang", "emotion", "event", "words")

    def __init__(self):
        self.text = ""
        self.tokens: List[str] = []
        self.timestamps: List[float] = []
        self.ys_log_probs: List[float] = []
        self.token_ids: List[int] = []
        self.frames: List[int] = []
        self.num_frames = 0
        self.lang = self.emotion = self.event = ""
        self.words: List = []

    def __str__(self):
        return json.dumps({"text": self.text, "timestamps": self.timestamps,
                           "tokens": self.tokens, "ys_log_probs": self.ys_log_probs})


class OfflineStream:
    """One utterance: samples accepted on the host until decoded (sherpa-onnx OfflineStream)."""

    def __init__(self, recognizer: "OfflineRecognizer"):
        self._rec = recognizer
        self._lib = recognizer._lib
        h = C.c_void_p()
        recognizer._check(self._lib.zasr_create_stream(recognizer._handle.handle, C.byref(h)))
        self._h = h
        self._result: Optional[OfflineRecognitionResult] = None
        self._fin = weakref.finalize(self, self._lib.zasr_destroy_stream, h)
        # f16x3: the samples stay on the host side too, so that a stream whose decode meets
        # the fp16 operand range can be re-decoded by the bf16x6 fallback engine
        self._samples: Optional[List[np.ndarray]] = [] if recognizer._can_fall_back else None
        self._delegate: Optional["OfflineStream"] = None  # the fallback engine's stream

    def accept_waveform(self, sample_rate: int, waveform) -> None:
        a = np.ascontiguousarray(np.asarray(waveform, dtype=np.float32).reshape(-1))
        fp = C.POINTER(C.c_float)
        self._rec._check(self._lib.zasr_stream_accept_waveform(
            self._h, int(sample_rate), a.ctypes.data_as(fp), int(a.shape[0])))
        if self._samples is not None:
            self._samples.append(a.copy())

    @property
    def result(self) -> OfflineRecognitionResult:
        if self._delegate is not None:
            return self._delegate.result
        if self._result is None:
            r = OfflineRecognitionResult()
            if self._lib.zasr_stream_is_decoded(self._h):
                self._result = r = self._rec._result_of(self._h)
            return r
        return self._result

    def as_json_string(self) -> str:
        """zasr_stream_result_json (SherpaOnnxGetOfflineStreamResultAsJson)."""
        if self._delegate is not None:
            return self._delegate.as_json_string()
        need = C.c_int64()
        self._lib.zasr_stream_result_json(self._h, None, 0, C.byref(need))
        if need.value <= 0:
            raise ZasrError(self._lib.zasr_last_error().decode())
        buf = C.create_string_buffer(int(need.value))
        self._rec._check(self._lib.zasr_stream_result_json(self._h, buf, len(buf), C.byref(need)))
        return buf.value.decode("utf-8")


def _load_symbols(path: str) -> dict:
    syms = {}
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 2:
                sym = parts[0]
                if sym.startswith("▁"):
                    sym = " " + sym[1:]
                syms[int(parts[-1])] = sym
    return syms


class OfflineRecognizer:
    """sherpa_onnx.OfflineRecognizer for transducer models, decoding on MI355X."""

    def __init__(self, model_dir: str, tokens: str, decoding_method: str = "greedy_search",
                 max_active_paths: int = 4, hotwords_file: str = "",
                 hotwords_score: float = 1.5, precision: Optional[str] = None,
                 device_id: Optional[int] = None):
        from zasr import asr_engine as ae
        if decoding_method not in ("greedy_search", "modified_beam_search"):
            raise ValueError(f"decoding_method must be greedy_search or modified_beam_search, "
                             f"got {decoding_method!r}")
        if not os.path.exists(tokens):
            raise FileNotFoundError(f"tokens file not found: {tokens}")
        seqs, scores = ae._hotword_token_lists(model_dir, hotwords_file, float(hotwords_score))
        dev = int(os.environ.get("ZASR_DEVICE", "0")) if device_id is None else int(device_id)
        prec = precision or os.environ.get("ZASR_PRECISION", ae.DEFAULT_PRECISION)
        self._handle = Recognizer(model_dir, decoding_method, int(max_active_paths),
                                  hotwords=seqs, hotword_scores=scores, device_id=dev,
                                  precision=prec)
        self._lib = self._handle.lib
        # the JSON result (zasr_stream_result_json) reads the same symbol table as .result
        self._handle._check(self._lib.zasr_set_tokens(self._handle.handle,
                                                      os.path.abspath(tokens).encode()))
        self._syms = _load_symbols(tokens)
        self._can_fall_back = prec == "f16x3"
        self._fallback: Optional["OfflineRecognizer"] = None
        self._ctor = (model_dir, tokens, decoding_method, int(max_active_paths), hotwords_file,
                      float(hotwords_score), dev)
        self.config = {"model_dir": model_dir, "tokens": tokens, "decoding_method": decoding_method,
                       "max_active_paths": int(max_active_paths), "precision": prec,
                       "num_hotwords": len(seqs)}

    @classmethod
    def from_transducer(cls, encoder: str, decoder: str, joiner: str, tokens: str,
                        num_threads: int = 1, sample_rate: int = 16000, feature_dim: int = 80,
                        decoding_method: str = "greedy_search", max_active_paths: int = 4,
                        hotwords_file: str = "", hotwords_score: float = 1.5,
                        blank_penalty: float = 0.0, provider: str = "cpu",
                        precision: Optional[str] = None, device_id: Optional[int] = None,
                        **unused) -> "OfflineRecognizer":
        """sherpa_onnx.OfflineRecognizer.from_transducer (streaming_asr.py:224-243).
        num_threads / provider / dither and the other CPU knobs do not apply to the GPU
        engine; sample_rate 16000, feature_dim 80 and blank_penalty 0 are the only values
        the engine implements (the reference passes exactly these)."""
        if int(sample_rate) != 16000 or int(feature_dim) != 80:
            raise ValueError("the MI355X engine decodes 16 kHz audio into 80-bin fbank features")
        if float(blank_penalty) != 0.0:
            raise ValueError("blank_penalty must be 0 (the reference applies none)")
        dirs = {os.path.dirname(os.path.abspath(p)) for p in (encoder, decoder, joiner)}
        if len(dirs) != 1:
            raise ValueError("encoder, decoder and joiner must be in one model directory")
        for p in (encoder, decoder, joiner):
            if not os.path.exists(p):
                raise FileNotFoundError(f"model file not found: {p}")
        return cls(dirs.pop(), tokens, decoding_method, max_active_paths, hotwords_file,
                   hotwords_score, precision, device_id)

    def _check(self, rc):
        if rc != 0:
            raise ZasrError(self._lib.zasr_last_error().decode())

    def create_stream(self, hotwords: Optional[str] = None) -> OfflineStream:
        if hotwords:
            raise ValueError("per-stream hotwords are not supported: pass hotwords_file to "
                             "from_transducer (the reference's usage)")
        return OfflineStream(self)

    def decode_stream(self, s: OfflineStream) -> None:
        try:
            self._check(self._lib.zasr_decode_stream(self._handle.handle, s._h))
        except ZasrError as e:
            self._fall_back(e, [s])
        s._result = None

    def decode_streams(self, ss: Sequence[OfflineStream]) -> None:
        """All streams in ONE batched GPU pass (SherpaOnnxDecodeMultipleOfflineStreams)."""
        ss = list(ss)
        arr = (C.c_void_p * max(len(ss), 1))(*[s._h.value for s in ss])
        try:
            self._check(self._lib.zasr_decode_streams(self._handle.handle, arr, len(ss)))
        except ZasrError as e:
            self._fall_back(e, ss)
        for s in ss:
            s._result = None

    # the stream path's form of zasr.binding.Recognizer._retry: an f16x3 decode whose encoder
    # output left the fp16 operand range (the engine reports it after draining its streams) is
    # redone by a bf16x6 engine of the same model, so the caller still gets the token-exact
    # result; each stream's result is then read from its twin on that engine
    def _fall_back(self, e: ZasrError, ss: Sequence[OfflineStream]) -> None:
        if not self._can_fall_back or "non-finite encoder output" not in str(e):
            raise e
        if self._fallback is None:
            import logging
            logging.getLogger("zasr").warning(
                "[zasr] f16x3 operand range exceeded; re-decoding with %s",
                Recognizer.FALLBACK_PRECISION)
            md, tok, method, beam, hwf, hws, dev = self._ctor
            self._fallback = OfflineRecognizer(md, tok, method, beam, hwf, hws,
                                               precision=Recognizer.FALLBACK_PRECISION,
                                               device_id=dev)
        twins = []
        for s in ss:
            t = self._fallback.create_stream()
            t.accept_waveform(16000, np.concatenate(s._samples) if s._samples
                              else np.zeros(0, np.float32))
            twins.append(t)
        self._fallback.decode_streams(twins)
        for s, t in zip(ss, twins):
            s._delegate = t

    def _result_of(self, h) -> OfflineRecognitionResult:
        lib = self._lib
        k = lib.zasr_stream_num_tokens(h)
        r = OfflineRecognitionResult()
        r.num_frames = int(lib.zasr_stream_num_frames(h))
        if k > 0:
            r.token_ids = np.ctypeslib.as_array(lib.zasr_stream_tokens(h), (k,)).tolist()
            r.frames = np.ctypeslib.as_array(lib.zasr_stream_frames(h), (k,)).tolist()
            r.ys_log_probs = np.ctypeslib.as_array(lib.zasr_stream_log_probs(h), (k,)).tolist()
        r.tokens = [self._syms.get(t, "") for t in r.token_ids]
        r.text = "".join(r.tokens)
        # frame shift 10 ms x subsampling factor 4, in float32 like sherpa-onnx
        r.timestamps = [float(np.float32(0.04) * np.float32(f)) for f in r.frames]
        return r

    @property
    def handle(self) -> Recognizer:
        return self._handle
