"""Shared inputs of the punctuation fixtures (tests/golden/make_golden_punct.py) and their
tests: a synthetic WordPiece vocabulary written as a model dir the reference's own
`GecBERTModel._get_indexer` loads with transformers' AutoTokenizer, a deterministic scripted
session (numpy function of the feeds, the onnxruntime `run(None, feeds)` surface), the word
generator of the transcripts and a recorder of every session call."""
from __future__ import annotations

import hashlib
import json
import os
from typing import Dict, List

import numpy as np

SPECIAL = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
SYLLABLES = ["xin", "chào", "các", "bạn", "tôi", "là", "người", "việt", "nam", "hôm", "nay",
             "trời", "đẹp", "quá", "chúng", "ta", "đi", "học", "làm", "việc", "ở", "hà", "nội",
             "thành", "phố", "hồ", "chí", "minh", "đại", "biểu", "quốc", "hội", "kính", "thưa",
             "đồng", "bảo", "vấn", "đề", "quy", "hoạch", "có", "nhiều", "giải", "pháp", "cảm",
             "ơn", "mời", "phát", "được", "không", "và", "của", "cho", "với", "một", "những"]
PIECES = ["##a", "##n", "##g", "##h", "##i", "##o", "##u", "##t", "##c", "##m", "##ng", "##nh",
          "a", "b", "c", "d", "đ", "e", "g", "h", "k", "l", "m", "n", "o", "p", "q", "r", "s"]
PUNCT = [".", ",", "?", ":"]
# 5 + 56 + 29 + 4 = 94 entries (< vibert_tiny's 100 ids before the added START token)
VOCAB = SPECIAL + SYLLABLES + PIECES + PUNCT


def write_model_dir(d: str) -> str:
    """vocab.txt + tokenizer_config.json: what AutoTokenizer.from_pretrained needs offline."""
    os.makedirs(d, exist_ok=True)
    assert len(set(VOCAB)) == len(VOCAB) <= 100
    with open(os.path.join(d, "vocab.txt"), "w", encoding="utf-8") as f:
        f.write("\n".join(VOCAB) + "\n")
    with open(os.path.join(d, "tokenizer_config.json"), "w") as f:
        json.dump({"tokenizer_class": "BertTokenizer", "do_lower_case": False}, f)
    return d


def words(n: int, seed: int) -> List[str]:
    """A transcript of n words: syllables in the vocab, ~1 in 10 out-of-vocab words built
    from letters (split into pieces or [UNK]), ~1 in 25 capitalised."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        r = rng.random()
        if r < 0.1:
            w = "".join(rng.choice(list("abcdghmnostu"), int(rng.integers(2, 6))))
        else:
            w = SYLLABLES[int(rng.integers(len(SYLLABLES)))]
        if rng.random() < 0.04:
            w = w.capitalize()
        out.append(w)
    return out


def pause_hints(n: int, seed: int) -> List[float]:
    rng = np.random.default_rng(seed)
    g = rng.choice([0.0, 0.05, 0.15, 0.3, 0.6, 1.2, 2.0], n, p=[.3, .2, .15, .12, .1, .08, .05])
    return [float(x) for x in g]


class ScriptedSession:
    """Logits of label k at word slot j = a hash of (first piece of word j, first piece of
    word j + 1, k, seed) scaled into [0, scale) (+ keep_bias on $KEEP): deterministic, depends
    on the text (appended punctuation changes the next iteration's predictions), exercises
    every label incl. the ones get_token_action rejects."""

    def __init__(self, seed: int, scale: float = 6.0, keep_bias: float = 0.0, n_labels: int = 15):
        self.seed, self.scale, self.keep_bias, self.n_labels = seed, scale, keep_bias, n_labels

    def _h(self, a, b, k):
        m = np.uint64(0xFFFFFFFF)
        h = (a.astype(np.uint64) * np.uint64(7919) + b.astype(np.uint64) * np.uint64(104729)
             + np.uint64(k) * np.uint64(1299709) + np.uint64(self.seed) * np.uint64(15485863)) & m
        h = ((h ^ (h >> np.uint64(13))) * np.uint64(0x5BD1E995)) & m
        return ((h ^ (h >> np.uint64(15))) % np.uint64(1024)).astype(np.float32) / np.float32(1024)

    def run(self, names, feeds):
        ids, off = feeds["input_ids"], feeds["input_offsets"]
        a = np.take_along_axis(ids, off, axis=1)
        nx = np.concatenate([off[:, 1:], np.zeros_like(off[:, :1])], axis=1)
        b = np.take_along_axis(ids, nx, axis=1)
        lg = np.stack([self._h(a, b, k) for k in range(self.n_labels)], -1) * np.float32(self.scale)
        lg[:, :, 0] += np.float32(self.keep_bias)
        dl = np.stack([self._h(a, b, 100 + k) for k in range(4)], -1) * np.float32(self.scale)
        return [lg.astype(np.float32), dl.astype(np.float32)]


def feeds_digest(feeds: Dict[str, np.ndarray]) -> str:
    h = hashlib.sha256()
    for k in ("input_ids", "attention_mask", "token_type_ids", "input_offsets"):
        v = np.ascontiguousarray(feeds[k], np.int64)
        h.update(k.encode() + str(v.shape).encode() + v.tobytes())
    return h.hexdigest()[:24]


class Recorder:
    """Wraps a session; keeps the digest of every run's feeds (the reference's mini-batches)."""

    def __init__(self, inner):
        self.inner, self.calls = inner, []

    def run(self, names, feeds):
        self.calls.append(feeds_digest(feeds))
        return self.inner.run(names, feeds)
