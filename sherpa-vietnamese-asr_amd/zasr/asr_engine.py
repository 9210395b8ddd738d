"""Drop-in `core/asr_engine.py` ASR surface backed by libzasr.so on MI355X.

This module lives under the `zasr` package (not under a `core` package) so that it never
shadows the reference's own `core` package: `zasr.dropin.install(core.asr_engine, ...)`
rebinds the reference module's hot-path names to the functions below.

Replaces the reference's onnxruntime + numpy hot path (`core/asr_engine.py:686-1326`)
with the same Python names, arguments and return shapes, so the reference's callers
(`TranscriberPipeline._run_pipeline` :2057-2494, `transcriber.py:26-34`,
`web_service/queue_manager.py:435-443`) keep working:

  get_ort()                      :686   import-compatible stub (no onnxruntime in this build)
  compute_fbank_ort(audio, sr)   :698   kaldi fbank -> HIP kernel
  _log_add(a, b)                 :724
  create_recognizer(...)         :903   dict with the same keys; sessions -> one zasr handle
  _ort_beam_search(rec, f, beam) :1023  (token_ids, frames, ys_log_probs, T, emit_stats)
  _compute_token_entropy(x, V)   :1159  accepts device stats (or a raw logits row)
  _finalize_word_entropy(w)      :1187
  decode_chunk(...)              :1209  same word dicts (BPE merge, timestamps, entropy)
  decode_chunks(...)             new    batched decode of many chunks in one GPU pass

Plan-ahead batching (how the reference's UNCHANGED caller reaches the batch pipeline): the
reference plans the whole file before decoding it (`TranscriberPipeline._run_pipeline`
:2137-2161 -- find_silent_regions over the concatenated speech, then ~30 s boundaries) and
then calls decode_chunk once per chunk from two worker threads (:2219-2237, :2326-2397).
zasr.dropin.install() wraps the module-level find_silent_regions so the plan is registered
(`register_plan`) the moment it is made; the first decode_chunk call that asks for a chunk
of a registered plan (a view into the planned signal at one of the plan's spans) decodes the
WHOLE plan in one batched GPU pass for that recognizer, and every later call -- from either
worker -- is served from those results.  Batched results equal per-chunk results bit for bit
(ragged batching, no padding), so the words are identical (tests/test_gpu_dropin.py).
Chunks that are not views of a planned signal (WPE-processed copies, other callers) take
the per-chunk path.  ZASR_PLAN_AHEAD=0 turns the routing off.

The search and the word post-processing stay semantically identical to the reference;
the arithmetic runs in libzasr (see DESIGN.md for precision modes and tolerances).
"""
from __future__ import annotations

import logging
import math
from functools import lru_cache
import os
import threading
import weakref
from typing import Dict, List, Optional, Sequence

import numpy as np

from zasr.binding import Recognizer

logger = logging.getLogger(__name__)

ROVER_MODEL_IDS = ["zipformer-30m-rnnt-6000h", "sherpa-onnx-zipformer-vi-2025-04-20"]
ROVER_MODEL_ID = "rover-voting"
BLANK_ID = 0
UNK_ID = 2
CONTEXT_SIZE = 2

# the precision create_recognizer (and zasr.offline) use unless told otherwise: f16x3, the
# fastest token-exact mode -- every f32 operand as two fp16 pieces (hi + lo * 2^-11), three
# fp16 MFMAs per product, ~2^-22 relative per product; operands must
# stay below fp16's 65504: a batch whose encoder output goes non-finite is re-decoded by a
# bf16x6 engine (three bf16 pieces: exact-f32 quality at f32 range; binding.Recognizer).
# bench.py reports it as parity_mode and times the drop-in stage in it; ZASR_PRECISION
# overrides
DEFAULT_PRECISION = "f16x3"

_recognizer_cache: Dict[tuple, dict] = {}
_cache_lock = threading.Lock()
_last_handle: Optional[Recognizer] = None
# the reference's core.asr_engine module once zasr.dropin.install() ran: its
# get_hotwords_config (core/config.py:385-408, imported at core/asr_engine.py top level)
# is where the hotword file and score come from, as in create_recognizer (:993-1003)
_HOST = None


def set_host_module(module) -> None:
    global _HOST
    _HOST = module


def get_ort():
    """The MI355X build has no onnxruntime; kept importable for `core/__init__.py:40-48`."""
    raise RuntimeError("onnxruntime is not part of the MI355X build: ASR runs in libzasr.so")


class TokenStats:
    """Per-token joiner-row statistics computed on device: entropy, sum p^(1/3), top1, top2.
    Stands in for the raw logits row the reference keeps per emitted token (:1125)."""
    __slots__ = ("entropy", "s3", "top1", "top2")

    def __init__(self, row):
        self.entropy, self.s3, self.top1, self.top2 = (float(x) for x in row)

    @staticmethod
    def rows(stats) -> List["TokenStats"]:
        """TokenStats of every row of an [n][4] float32 array (one tolist(): the same Python
        floats as float() of each element, without the per-element numpy scalars)."""
        out = []
        for e, s3, t1, t2 in np.asarray(stats, np.float32).reshape(-1, 4).tolist():
            t = TokenStats.__new__(TokenStats)
            t.entropy, t.s3, t.top1, t.top2 = e, s3, t1, t2
            out.append(t)
        return out


def _default_handle() -> Recognizer:
    if _last_handle is None:
        raise RuntimeError("compute_fbank_ort needs a recognizer: call create_recognizer first")
    return _last_handle


def compute_fbank_ort(audio, sr=16000):
    """80-bin kaldi log-mel fbank (reference :698-721) computed by the HIP fbank kernel."""
    if sr != 16000:
        raise ValueError("only 16 kHz input is supported (reference resamples on load)")
    feats = _default_handle().fbank(np.asarray(audio, dtype=np.float32))
    _note_features(feats, audio)
    return feats


def _log_add(a, b):
    if a < b:
        a, b = b, a
    diff = b - a
    return a if diff < -36.0 else a + np.log1p(np.exp(diff))


def clear_model_cache(which="all"):
    """Drops this build's recognizer cache (reference :743-768, the 'recognizer' part).  The
    native engines are released by reference count: copies of a recognizer dict
    (`dict(recognizer_2)`, core/asr_engine.py:2306) share the handle, and the last one to
    go frees it (Recognizer.__del__).  After install() the reference's own clear_model_cache
    still runs for the punctuation restorer and diarizer (zasr.dropin)."""
    global _last_handle
    if which in ("all", "recognizer"):
        with _cache_lock:
            _recognizer_cache.clear()
            _last_handle = None


def _onnx_file(model_path: str, pattern: str) -> Optional[str]:
    """The reference's find_file (core/asr_engine.py:913-920): the first entry starting with
    `pattern` and ending in .onnx without "int8" in its name, else the first such file."""
    try:
        names = os.listdir(model_path)
    except OSError:
        return None
    files = [f for f in names if f.startswith(pattern) and f.endswith(".onnx")]
    floats = [f for f in files if "int8" not in f]
    if floats:
        return os.path.join(model_path, floats[0])
    return os.path.join(model_path, files[0]) if files else None


def model_files_present(model_path: str) -> bool:
    """tokens.txt plus either this build's config.json + model.safetensors or the reference's
    encoder-/decoder-/joiner-*.onnx set (libzasr reads their initializers, csrc/onnx_io.cpp)."""
    if not os.path.exists(os.path.join(model_path, "tokens.txt")):
        return False
    if all(os.path.exists(os.path.join(model_path, f)) for f in ("config.json", "model.safetensors")):
        return True
    return all(_onnx_file(model_path, p) for p in ("encoder-", "decoder-", "joiner-"))


def _load_tokens(path: str) -> Dict[int, str]:
    id2token = {}
    with open(path, "r", encoding="utf-8") as f:
        for line in f:
            parts = line.strip().split()
            if len(parts) >= 2:
                id2token[int(parts[-1])] = parts[0]
    return id2token


def _hotword_token_lists(model_path: str, hotwords_file: Optional[str], default_score: float):
    """Hotword phrases -> token ids with the model's sentencepiece model (host side, as in
    core/hotword_context.py:225-259).  Without bpe.model no graph is built (reference :999)."""
    bpe = os.path.join(model_path, "bpe.model")
    if not hotwords_file or not os.path.exists(bpe):
        return [], []
    from zasr.hotword_context import parse_hotwords_file
    phrases = parse_hotwords_file(hotwords_file, default_score)
    if not phrases:
        return [], []
    import sentencepiece as spm
    sp = spm.SentencePieceProcessor()
    sp.load(bpe)
    seqs, scores = [], []
    for text, score in phrases:
        ids = sp.encode(text, out_type=int)
        if ids:
            seqs.append(ids)
            scores.append(score)
    return seqs, scores


def _hotword_config(model_path: str):
    """(hotwords_file, hotwords_score) the way the reference's create_recognizer finds them
    (:993-1003): `get_hotwords_config(model_path)` of the installed reference module.  The
    env vars ZASR_HOTWORDS_FILE / ZASR_HOTWORDS_SCORE override it (standalone use)."""
    env_file = os.environ.get("ZASR_HOTWORDS_FILE")
    if env_file is not None:
        return env_file, float(os.environ.get("ZASR_HOTWORDS_SCORE", 1.5))
    get_cfg = getattr(_HOST, "get_hotwords_config", None) if _HOST is not None else None
    if get_cfg is None:
        return "", 1.5
    try:
        cfg = get_cfg(model_path) or {}
    except Exception as e:  # the reference logs and continues without a graph (:1002-1003)
        print(f"[Hotwords] Failed to build context graph: {e}")
        return "", 1.5
    return cfg.get("hotwords_file", ""), float(cfg.get("hotwords_score", 1.5))


def create_recognizer(model_path, cpu_threads=4, max_active_paths=8, execution_provider="cpu",
                      hotwords=None, device_id=None, precision=None):
    """Load (or reuse) a recognizer for `model_path` (reference :903-1020).

    Model directory: tokens.txt + either config.json + model.safetensors (zasr/model.py) or the
    reference's encoder-/decoder-/joiner-*.onnx files (read by libzasr, non-int8 preferred like
    :913-928).  Raises FileNotFoundError when files are missing, like the reference (:927-928).
    Hotwords: the reference's hotword config (see _hotword_config) tokenized with the model's
    bpe.model; `hotwords` may be (token_id_lists, scores) to bypass the file + bpe route.
    """
    provider_policy = str(execution_provider or "cpu").lower()
    dev = int(os.environ.get("ZASR_DEVICE", "0")) if device_id is None else int(device_id)
    prec = precision or os.environ.get("ZASR_PRECISION", DEFAULT_PRECISION)
    # cpu_threads / execution_provider do not change the GPU engine, so they are not part of
    # the key: the reference re-creates the recognizer with the worker thread count before its
    # two workers start (:2290-2307), which must not load a second copy of the model
    key = (os.path.normpath(model_path), max_active_paths, dev, prec,
           None if hotwords is None else repr(hotwords))
    global _last_handle
    with _cache_lock:
        if key in _recognizer_cache:
            _last_handle = _recognizer_cache[key]["handle"]
            return _recognizer_cache[key]
        tokens_path = os.path.join(model_path, "tokens.txt")
        if not model_files_present(model_path):
            raise FileNotFoundError(f"Thiếu file model trong: {model_path}")
        if hotwords is not None:
            seqs, scores = [list(map(int, s)) for s in hotwords[0]], list(map(float, hotwords[1]))
        else:
            hw_file, hw_score = _hotword_config(model_path)
            seqs, scores = _hotword_token_lists(model_path, hw_file, hw_score)
        handle = Recognizer(model_path, "modified_beam_search", int(max_active_paths),
                            hotwords=seqs, hotword_scores=scores, device_id=dev, precision=prec)
        info = {"actual_provider": f"MI355X:HIP(device {dev}, {prec})"}
        rec = {
            "handle": handle,
            "id2token": _load_tokens(tokens_path),
            "vocab_size": handle.vocab_size,
            "max_active_paths": int(max_active_paths),
            "model_path": model_path,
            "dec_cache": {},
            "context_graph": {"num_phrases": len(seqs)} if seqs else None,
            "provider_info": {"encoder": info, "decoder": info, "joiner": info},
        }
        _recognizer_cache[key] = rec
        _last_handle = handle
        return rec


def _ort_beam_search(recognizer, features, beam_size=8):
    """Modified beam search over one chunk's features (reference :1023-1153).
    Returns (token_ids, frames, ys_log_probs, T, emit_stats)."""
    r = recognizer["handle"].decode_features([np.asarray(features, np.float32)],
                                            beam=int(beam_size))[0]
    return (r.token_ids.tolist(), r.frames.tolist(), r.log_probs.tolist(), int(r.T),
            [TokenStats(s) for s in r.stats])


@lru_cache(maxsize=64)
def _entropy_norms(V):
    """(max entropy, Tsallis-1/3 maximum) of a vocabulary (reference :1161-1165)."""
    alpha = 1.0 / 3.0
    max_entropy = math.log(V) if V > 1 else 1.0
    ts_max = (1.0 / (alpha - 1.0)) * (1.0 - V ** (1.0 - alpha)) if V > 1 else 1.0
    return max_entropy, ts_max


def _compute_token_entropy(raw_logits, V):
    """Entropy metrics of one emitted token (reference :1159-1181).  Accepts the device
    TokenStats (normal path) or a raw logits row (computed as the reference does)."""
    max_entropy, ts_max = _entropy_norms(V)
    alpha = 1.0 / 3.0
    if isinstance(raw_logits, TokenStats):
        entropy, s3, top1, top2 = raw_logits.entropy, raw_logits.s3, raw_logits.top1, raw_logits.top2
    else:
        z = np.asarray(raw_logits, np.float32)
        p = np.exp(z - np.max(z))
        p /= np.sum(p)
        entropy = -float(np.sum(p * np.log(p + 1e-30)))
        s3 = float(np.sum(p ** alpha))
        srt = np.sort(p)[::-1]
        top1 = float(srt[0])
        top2 = float(srt[1]) if len(srt) > 1 else 1e-10
    tsallis = (1.0 / (alpha - 1.0)) * (1.0 - s3)
    return {
        "tsallis_norm": round(float(tsallis / ts_max if ts_max > 0 else 0.0), 4),
        "margin": round(top1 - top2, 4),
        "entropy_norm": round(entropy / max_entropy, 4),
        "top1_prob": top1,
    }


_ENTROPY_FALLBACK = {"tsallis_norm": 0, "margin": 1, "entropy_norm": 0, "top1_prob": 1.0}


def _np_mean(xs):
    """np.mean of a list of Python floats, bit for bit: numpy's float64 pairwise sum
    (sequential below 8 elements; eight interleaved partial sums combined as
    ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail, up to its 128-element block; larger
    lists go to numpy) divided by the count -- without the array round trip per word."""
    n = len(xs)
    if n < 8:
        s = 0.0
        for x in xs:
            s += x
        return s / n
    if n > 128:
        return float(np.mean(xs))
    r = list(xs[:8])
    i = 8
    while i + 8 <= n:
        for k in range(8):
            r[k] += xs[i + k]
        i += 8
    s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
    for x in xs[i:]:
        s += x
    return s / n


def _finalize_word_entropy(w):
    """BPE-level -> word-level aggregation (reference :1187-1206)."""
    probs = w.pop("probs")
    w["prob"] = sum(probs) / len(probs)
    ents = w.pop("_ents", [])
    if ents:
        w["tsallis_max"] = round(float(max(e["tsallis_norm"] for e in ents)), 4)
        w["margin_min"] = round(float(min(e["margin"] for e in ents)), 4)
        w["entropy_norm"] = round(_np_mean([e["entropy_norm"] for e in ents]), 4)
        confs = [e["margin"] * (1.0 - e["tsallis_norm"]) for e in ents]
        w["_conf"] = round(float(sum(confs) / len(confs)), 4)
    else:
        w["tsallis_max"] = w["margin_min"] = w["entropy_norm"] = w["_conf"] = None


def _words_from_search(id2token, V, n_samples, time_offset, token_ids, frames, log_probs, T,
                       emit_stats):
    """BPE -> word dicts with timestamps, probabilities and entropy (reference :1227-1326)."""
    if not token_ids:
        return []
    pieces = [id2token.get(t, "") for t in token_ids]
    chunk_dur = n_samples / 16000.0
    ts = [f / T * chunk_dur for f in frames] if T > 0 else []
    if not ts:
        return []
    avg = (ts[-1] - ts[0]) / (len(ts) - 1) if len(ts) >= 2 else 0.08
    ents = [_compute_token_entropy(emit_stats[j], V) if j < len(emit_stats) else _ENTROPY_FALLBACK
            for j in range(len(token_ids))]
    words: List[dict] = []
    cur = None
    for j, (t0, piece) in enumerate(zip(ts, pieces)):
        text = piece.lower()
        t1 = ts[j + 1] if j + 1 < len(ts) else t0 + avg
        prob = math.exp(log_probs[j]) if j < len(log_probs) else 1.0
        ent = ents[j]
        starts_word = text.startswith(" ") or text.startswith("▁")
        if starts_word or cur is None:
            if cur is not None:
                _finalize_word_entropy(cur)
                words.append(cur)
            cur = {"text": text.lstrip(" ").lstrip("▁") if starts_word else text,
                   "start": t0 + time_offset, "end": t1 + time_offset,
                   "local_start": t0, "local_end": t1, "last_bpe_start": t0 + time_offset,
                   "probs": [prob], "_ents": [ent] if ent else []}
        else:
            cur["text"] += text
            cur["end"] = t1 + time_offset
            cur["local_end"] = t1
            cur["last_bpe_start"] = t0 + time_offset
            cur["probs"].append(prob)
            if ent:
                cur["_ents"].append(ent)
    if cur is not None:
        _finalize_word_entropy(cur)
        words.append(cur)
    if words:
        words[0]["_chunk_bpe_tokens"] = list(pieces)
        words[0]["_chunk_bpe_timestamps_local"] = list(ts)
    for i, w in enumerate(words):
        end = w["last_bpe_start"] + avg
        if i + 1 < len(words):
            end = min(end, words[i + 1]["start"])
        w["end"] = end
        w["local_end"] = end - time_offset
        del w["last_bpe_start"]
    return words


try:  # the same post-processing in C (csrc/words_ext.c); Python >= 3.12 sums floats with
    # compensation (sum()), which the C twin does not restate: the Python version runs there
    import sys as _sys
    from zasr import _zasr_words
    if _sys.version_info >= (3, 12):
        _zasr_words = None
except ImportError:  # pragma: no cover - built by __graft_entry__.build() / make
    _zasr_words = None

_tok_tables: Dict[int, tuple] = {}


def _token_tables(id2token):
    """(pieces, lowered) lists indexed by token id for the C word builder: id2token.get(t, "")
    and its .lower(), built once per vocabulary."""
    ent = _tok_tables.get(id(id2token))
    if ent is None or ent[0] is not id2token or ent[1] != len(id2token):
        hi = max((k for k in id2token if isinstance(k, int)), default=-1)
        pieces = [id2token.get(i, "") for i in range(hi + 1)]
        ent = (id2token, len(id2token), pieces, [p.lower() for p in pieces])
        _tok_tables[id(id2token)] = ent
    return ent[2], ent[3]


def result_words(recognizer, r, n_samples: int, time_offset: float):
    """Word dicts of one device search result (reference :1227-1326): the tail of
    decode_chunk, shared by decode_chunk / decode_chunks / the ROVER path.  Runs in the C
    extension when it is built (identical dicts, tests/test_words_ext.py), else in Python."""
    if _zasr_words is not None:
        pieces, lowered = _token_tables(recognizer["id2token"])
        return _zasr_words.words_from_search(
            pieces, lowered, int(recognizer["vocab_size"]), int(n_samples), float(time_offset),
            np.ascontiguousarray(r.token_ids, np.int32), np.ascontiguousarray(r.frames, np.int32),
            np.ascontiguousarray(r.log_probs, np.float64), int(r.T),
            np.ascontiguousarray(r.stats, np.float32))
    return _words_from_search(recognizer["id2token"], recognizer["vocab_size"], n_samples,
                              time_offset, r.token_ids.tolist(), r.frames.tolist(),
                              r.log_probs.tolist(), int(r.T), TokenStats.rows(r.stats))


# ------------------------------------------------------------------ plan-ahead batching
PLAN_BATCH_CHUNKS = 256  # chunks per batch of the plan's decode (~2 h of audio)
FRAME_LEN = 160          # find_silent_regions' 10 ms frame at 16 kHz (:526)
SILENCE_THRESHOLD = 0.01  # its defaults (:521)
MIN_SILENCE_SEC = 0.3


class _PlannedSignal:
    """A signal the reference's planner cut into chunks.  Holds the signal weakly (the
    pipeline owns it), the signal's HBM copy when the GPU silence detector uploaded it, and
    per recognizer handle and beam one decode of every chunk of the plan: started in the
    background the moment the plan is registered (for the recognizers already loaded, which
    the reference creates before it plans, :2041-2057), or on the first chunk asked for."""

    def __init__(self, audio: np.ndarray, plan, d_audio=None):
        # when the pipeline drops the signal, the entry goes with it (its HBM copy and the
        # plan's results): _prune_planned runs from the weakref callback
        self.ref = weakref.ref(audio, lambda _r: _prune_planned())
        self.ptr = audio.__array_interface__["data"][0]
        self.n = int(audio.shape[0])
        self.plan = [(int(s), int(e)) for s, e, _ in plan if int(e) > int(s)]
        self.spans = set(self.plan)
        self.d_audio = d_audio
        self.lock = threading.Lock()
        self.jobs = weakref.WeakKeyDictionary()  # handle -> {beam: _PlanDecode}
        self.running = 0

    def alive(self) -> bool:
        return self.ref() is not None

    def _decode(self, handle, beam):
        """Every chunk of the plan through the batch pipeline: from the HBM copy when there
        is one (no second upload), else from the host signal."""
        audio = self.ref()
        if audio is None:
            return None
        res = {}
        sizes = [min(PLAN_BATCH_CHUNKS, len(self.plan) - i)
                 for i in range(0, len(self.plan), PLAN_BATCH_CHUNKS)]
        d_audio = self.d_audio
        if d_audio is not None and getattr(handle, "device_id", None) == d_audio.device.index:
            out = handle.decode_device_batches(d_audio.data_ptr(), [s for s, _ in self.plan],
                                               [e - s for s, e in self.plan], sizes, beam=beam)
            res.update(zip(self.plan, out))
        else:
            for i in range(0, len(self.plan), PLAN_BATCH_CHUNKS):
                part = self.plan[i:i + PLAN_BATCH_CHUNKS]
                res.update(zip(part, handle.decode([audio[s:e] for s, e in part], beam=beam)))
        return res

    def start(self, handle, beam: int) -> "_PlanDecode":
        with self.lock:
            per = self.jobs.get(handle)
            if per is None:
                per = self.jobs[handle] = {}
            job = per.get(beam)
            if job is None:
                job = per[beam] = _PlanDecode(self, handle, beam)
                self.running += 1
        return job

    def job_done(self) -> None:
        """A plan decode finished: once none is running, the signal's HBM copy is released
        (a decode started later for another recognizer reads the host signal instead)."""
        with self.lock:
            self.running -= 1
            if self.running == 0:
                self.d_audio = None

    def result(self, handle, beam: int, span):
        """The plan's result for `span`, or None when the plan's decode failed (logged once;
        the caller then decodes the chunk on its own, as without plan-ahead)."""
        res = self.start(handle, beam).wait()
        return None if res is None else res.get(span)


class _PlanDecode:
    """One background decode of a plan for (handle, beam); wait() returns its results (the
    ctypes call releases the GIL, so the caller's own work runs beside the GPU decode)."""

    def __init__(self, sig: _PlannedSignal, handle, beam: int):
        self.res, self.err = None, None
        self.lock, self.logged = threading.Lock(), False
        self.t_start = self.t_end = None  # perf_counter() around the decode (bench phase split)
        self.thread = threading.Thread(target=self._run, args=(weakref.ref(sig), handle, beam),
                                       name="zasr-plan-decode", daemon=True)
        self.thread.start()

    def _run(self, sig_ref, handle, beam):
        import time
        self.t_start = time.perf_counter()
        sig = sig_ref()
        try:
            self.res = sig._decode(handle, beam) if sig is not None else None
        except BaseException as e:  # reported once by wait(); the chunks fall back
            self.err = e
        finally:
            self.t_end = time.perf_counter()
            if sig is not None:
                sig.job_done()
            del sig

    def wait(self):
        """The plan's results, or None when its decode failed.  Plan-ahead is an optimisation
        and must never break the caller (zasr.dropin): a failure (e.g. out of HBM on a long
        file while other stages hold memory) is logged once and every chunk of the plan takes
        the per-chunk path, which may still succeed."""
        self.thread.join()
        if self.err is not None:
            with self.lock:
                if not self.logged:
                    self.logged = True
                    logger.warning(f"[zasr] plan decode failed, chunks decode one by one: "
                                   f"{self.err!r}")
            return None
        return self.res


_plan_lock = threading.RLock()  # re-entered by the signal weakref callback
_planned: List[_PlannedSignal] = []
_feat_src: Dict[int, tuple] = {}  # id(features) -> (weakref(features), chunk data ptr, samples)


def _plan_ahead_on() -> bool:
    return os.environ.get("ZASR_PLAN_AHEAD", "1") != "0"


def _is_f32_vector(a) -> bool:
    return (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.ndim == 1
            and a.strides == (4,))


def _loaded_handles():
    """(handle, beam) of the recognizers the cache holds (the reference creates its one --
    or, for ROVER, two -- recognizers before it plans); none when more are cached."""
    with _cache_lock:
        recs = list(_recognizer_cache.values())
    out, seen = [], set()
    for r in recs:
        h = r["handle"]
        if id(h) not in seen:
            seen.add(id(h))
            out.append((h, int(r.get("max_active_paths", 8)), r.get("model_path", "")))
    return out if len(out) <= 2 else []


def _eager_handles():
    """The recognizers whose plan decode starts at registration: the one used last (the
    reference creates it right before planning, :2041-2057) and, when the two cached models
    are the ROVER pair (ROVER_MODEL_IDS, :2018-2047), both.  Any other cached recognizer (an
    earlier model still in the cache) starts its decode on its first planned chunk instead."""
    loaded = _loaded_handles()
    names = {os.path.basename(os.path.normpath(p)) for _, _, p in loaded}
    if len(loaded) == 2 and names == set(ROVER_MODEL_IDS):
        return [(h, b) for h, b, _ in loaded]
    return [(h, b) for h, b, _ in loaded if h is _last_handle][:1]


def _prune_planned() -> None:
    with _plan_lock:
        _planned[:] = [p for p in _planned if p.alive()]


def register_plan(audio, plan, d_audio=None, start: bool = True) -> bool:
    """Remember that `audio` (the signal the planner worked on) is cut into `plan`
    [(start, end, overlap)]; chunks decode_chunk later receives as views of it at those spans
    are served from one batched decode of the plan, started now for the loaded recognizers.
    `d_audio`: the signal's HBM copy (a torch tensor), when the GPU planner made one.  Keeps
    the last few signals (weakly)."""
    if not _plan_ahead_on() or not _is_f32_vector(audio) or not plan:
        return False
    sig = _PlannedSignal(audio, plan, d_audio)
    with _plan_lock:
        _planned[:] = [p for p in _planned if p.alive()][-3:] + [sig]
    if start:
        for h, beam in _eager_handles():
            sig.start(h, beam)
    return True


def register_plan_from_regions(audio, regions, best_split_fn=None, d_audio=None,
                               start: bool = True) -> bool:
    """The find_silent_regions hook: the plan the reference builds from these regions
    (:2141-2161, zasr.plan.plan_from_regions with the reference's own find_best_split_point)."""
    from zasr.plan import plan_from_regions
    if not _is_f32_vector(audio):
        return False
    return register_plan(audio, plan_from_regions(int(audio.shape[0]), regions, best_split_fn),
                         d_audio, start)


def _gpu_planner_on() -> bool:
    return _plan_ahead_on() and os.environ.get("ZASR_GPU_PLANNER", "1") != "0"


def silent_regions_device(audio: np.ndarray, device_id: int = 0):
    """find_silent_regions (:521-554) with its defaults, on the GPU: the signal goes to HBM
    once (it stays there for the plan's decode), zasr_silence_flags evaluates every 10 ms
    frame's RMS < 0.01 exactly as numpy's float32 does, and the regions are built from the
    flags on the host (zasr.plan.regions_from_flags).  Returns (regions, device tensor)."""
    import torch
    from zasr.binding import silence_flags
    from zasr.plan import regions_from_flags
    n = int(audio.shape[0])
    nf = n // FRAME_LEN
    dev = torch.device("cuda", int(device_id))
    d = torch.from_numpy(audio).to(dev)
    if nf == 0:
        return [], d
    flags = torch.empty(nf, dtype=torch.uint8, device=dev)
    silence_flags(d.data_ptr(), n, FRAME_LEN, SILENCE_THRESHOLD, flags.data_ptr(),
                  torch.cuda.current_stream(dev).cuda_stream)
    return regions_from_flags(flags.cpu().numpy().astype(bool), FRAME_LEN, n, MIN_SILENCE_SEC), d


def plan_ahead_regions(audio, best_split_fn=None, start: bool = True):
    """The drop-in's find_silent_regions for the planner's default-argument calls
    (:2139, :2183): the regions from the GPU silence detector (bit-identical to the
    reference's), with the plan built from them registered and its decode started (unless
    `start` is False: the caller's chunks will not be views of this signal, e.g. WPE).  None
    when the route does not apply (then the reference's own function runs)."""
    if not _gpu_planner_on() or not _is_f32_vector(audio) or not audio.flags.writeable:
        return None
    handles = _eager_handles() or [(h, b) for h, b, _ in _loaded_handles()]
    dev = handles[0][0].device_id if handles else int(os.environ.get("ZASR_DEVICE", "0"))
    regions, d = silent_regions_device(audio, dev)
    register_plan_from_regions(audio, regions, best_split_fn, d_audio=d if start else None,
                               start=start)
    return regions


def _planned_span(chunk):
    """(planned signal, (start, end)) when `chunk` is a view of a registered signal at one of
    its plan's spans, else None."""
    if not _is_f32_vector(chunk) or chunk.shape[0] == 0:
        return None
    p = chunk.__array_interface__["data"][0]
    with _plan_lock:
        sigs = list(_planned)
    for sig in reversed(sigs):
        if sig.ref() is None:
            continue
        off = p - sig.ptr
        if off >= 0 and off % 4 == 0:
            span = (off // 4, off // 4 + int(chunk.shape[0]))
            if span in sig.spans:
                return sig, span
    return None


def _note_features(feats, audio) -> None:
    """compute_fbank_ort output: remember which chunk it came from, so decode_chunk with these
    precomputed features (the ROVER path, :2346-2350) can still use the plan's batch results
    (the batch computes the same fbank kernel on the same samples)."""
    if not _plan_ahead_on() or not _is_f32_vector(audio):
        return
    key = id(feats)

    def drop(_, k=key):
        _feat_src.pop(k, None)
    _feat_src[key] = (weakref.ref(feats, drop), audio.__array_interface__["data"][0],
                      int(audio.shape[0]))


def _planned_result(handle, beam, audio_chunk, precomputed_features):
    if not _plan_ahead_on():
        return None
    if precomputed_features is not None:
        src = _feat_src.get(id(precomputed_features))
        if (src is None or src[0]() is not precomputed_features or not _is_f32_vector(audio_chunk)
                or src[1] != audio_chunk.__array_interface__["data"][0]
                or src[2] != audio_chunk.shape[0]):
            return None
    hit = _planned_span(audio_chunk)
    if hit is None:
        return None
    return hit[0].result(handle, beam, hit[1])


def decode_chunk(recognizer, audio_chunk, time_offset=0.0, precomputed_features=None):
    """Decode one chunk into merged word dicts (reference :1209-1326).  A chunk of a
    registered plan is served from the plan's batched decode (see the module docstring)."""
    beam = recognizer.get("max_active_paths", 8)
    h: Recognizer = recognizer["handle"]
    r = _planned_result(h, beam, audio_chunk, precomputed_features)
    if r is None:
        if precomputed_features is not None:
            feats = np.asarray(precomputed_features, np.float32)
            if feats.shape[0] == 0:
                return []
            r = h.decode_features([feats], beam=beam)[0]
        else:
            a = np.asarray(audio_chunk, np.float32)
            if a.shape[0] == 0:
                return []
            r = h.decode([a], beam=beam)[0]
    return result_words(recognizer, r, len(audio_chunk), time_offset)


def decode_chunks(recognizer, chunks: Sequence[np.ndarray], time_offsets: Sequence[float],
                  precomputed_features: Optional[Sequence[np.ndarray]] = None):
    """Batched decode_chunk: every chunk goes through one GPU pass (fbank, encoder, search).

    Under an initialised torch.distributed group (one process per GPU) each rank decodes its
    LPT share of the chunks and every rank receives all word lists in chunk order
    (zasr.shard.decode_sharded; host-side gather, no GPU collective)."""
    from zasr.shard import decode_sharded
    beam = recognizer.get("max_active_paths", 8)
    h: Recognizer = recognizer["handle"]
    items = list(zip(chunks, time_offsets,
                     precomputed_features if precomputed_features is not None else [None] * len(chunks)))

    def run(part):
        if not part:
            return []
        if precomputed_features is not None:
            res = h.decode_features([np.asarray(f, np.float32) for _, _, f in part], beam=beam)
        else:
            res = h.decode([np.asarray(c, np.float32) for c, _, _ in part], beam=beam)
        return [result_words(recognizer, r, len(c), off) for (c, off, _), r in zip(part, res)]

    return decode_sharded(run, items, lengths=[len(c) for c in chunks])
