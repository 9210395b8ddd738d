"""Generate the punctuation fixtures by running the REFERENCE's own GecBERTModel and
ImprovedPunctuationRestorer (build container only; the reference never travels):

    python tests/golden/make_golden_punct.py

* `onnxruntime` (absent here) is replaced in sys.modules by a stub whose InferenceSession
  returns the session object chosen per case; everything else is the reference's code:
  GecBERTModel.__init__ with the restorer's arguments (core/punctuation_restorer_improved.py:
  35-47), its Vocabulary.from_files on a temp COPY of the reference's vocabulary/ (from_files
  takes a lock file inside the directory it reads), its _get_indexer (transformers'
  AutoTokenizer on a synthetic WordPiece vocab.txt, tests/punct_sessions.py), handle_batch,
  and the restorer's restore/_post_process (the restorer object is made with object.__new__
  so its constructor's reference-relative paths are not touched).
* sessions: tests/punct_sessions.ScriptedSession (a numpy function of the feeds) and the
  ViBERT oracle (oracle/vibert.py, the tiny config, zasr.vibert.synth_weights with the
  classifier scaled so that labels other than $KEEP win), each wrapped in a Recorder that
  keeps a digest of every run's feeds.

Writes tests/golden/punct_cases.json: per case the inputs, the session spec, the reference's
output text and the digests of its session runs (the mini-batched feeds of every iteration).
"""
from __future__ import annotations

import contextlib
import importlib.machinery
import io
import json
import os
import shutil
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
REF = "/root/reference"
ORACLE_SCALE = 40.0


def oracle_session(seed: int):
    from oracle.vibert import VibertOracle
    from zasr.vibert import synth_weights, vibert_tiny
    cfg = vibert_tiny()
    w = synth_weights(cfg, seed)
    w["classifier.weight"] = w["classifier.weight"] * np.float32(ORACLE_SCALE)
    o = VibertOracle(cfg, w)

    class S:
        margins = []

        def run(self, names, feeds):
            lg, dl = o.run(feeds["input_ids"], feeds["attention_mask"], feeds["token_type_ids"],
                           feeds["input_offsets"])
            p = np.exp(lg - lg.max(-1, keepdims=True))
            p /= p.sum(-1, keepdims=True)
            p[:, :, 0] += 0.3
            s = np.sort(p, -1)
            S.margins.append(float((s[..., -1] - s[..., -2]).min()))
            return [lg, dl]
    return S()


def make_session(spec):
    from punct_sessions import ScriptedSession
    if spec["kind"] == "scripted":
        return ScriptedSession(spec["seed"], spec["scale"], spec["keep_bias"])
    return oracle_session(spec["seed"])


def cases():
    from punct_sessions import pause_hints, words
    sc = lambda seed, scale=6.0, kb=0.0: {"kind": "scripted", "seed": seed, "scale": scale,
                                           "keep_bias": kb}
    out = []
    for i, n in enumerate([0, 2, 3, 10, 56, 57, 95, 96, 150, 333]):
        out.append({"kind": "restore", "session": sc(10 + i, 6.0, 0.5 * (i % 3)),
                    "text": " ".join(words(n, 100 + i)) if n else "", "pause_hints": None})
    for i, n in enumerate([40, 120, 260]):
        out.append({"kind": "restore", "session": sc(40 + i), "text": " ".join(words(n, 200 + i)),
                    "pause_hints": pause_hints(n, 300 + i)})
    w = words(140, 77)
    for k in range(5, 140, 11):
        w[k] = "."
    out.append({"kind": "restore", "session": sc(50), "text": " ".join(w), "pause_hints": None})
    out.append({"kind": "restore", "session": sc(51, 6.0, -1.0),
                "text": " ".join(x.upper() if j % 4 == 0 else x for j, x in enumerate(words(70, 78))),
                "pause_hints": None})
    texts = [" ".join(words(n, 400 + j)) for j, n in
             enumerate([100, 220, 180, 2, 150, 210, 0, 190, 160, 205, 130, 215, 60])]
    out.append({"kind": "batch", "session": sc(60), "texts": texts, "pause_hints": None})
    hints = [pause_hints(len(t.split()), 500 + j) for j, t in enumerate(texts)]
    out.append({"kind": "batch", "session": sc(61, 5.0, 0.3), "texts": texts, "pause_hints": hints})
    for j, n in enumerate([12, 70, 150]):
        out.append({"kind": "restore", "session": {"kind": "oracle", "seed": 600 + j},
                    "text": " ".join(words(n, 700 + j)), "pause_hints": None})
    out.append({"kind": "batch", "session": {"kind": "oracle", "seed": 610},
                "texts": texts[:6], "pause_hints": None})
    return out


def main():
    sys.path[:0] = [TESTS, REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd"), REF]
    from punct_sessions import Recorder, write_model_dir
    current = {}
    ort = types.ModuleType("onnxruntime")
    ort.__spec__ = importlib.machinery.ModuleSpec("onnxruntime", None)  # torch._dynamo probes it

    class SessionOptions:
        pass
    ort.SessionOptions = SessionOptions
    ort.GraphOptimizationLevel = types.SimpleNamespace(ORT_ENABLE_ALL=99)
    ort.InferenceSession = lambda *a, **k: current["session"]
    sys.modules["onnxruntime"] = ort
    with contextlib.redirect_stdout(io.StringIO()):
        from core.gec_model import GecBERTModel
        from core.punctuation_restorer_improved import ImprovedPunctuationRestorer
    assert os.path.realpath(sys.modules["core.gec_model"].__file__).startswith(REF)
    tmp = tempfile.mkdtemp()
    vocab = os.path.join(tmp, "vocabulary")
    os.makedirs(vocab)
    for f in ("labels.txt", "d_tags.txt", "non_padded_namespaces.txt"):
        shutil.copy(os.path.join(REF, "vocabulary", f), vocab)
    model = write_model_dir(os.path.join(tmp, "vibert-capu"))
    open(os.path.join(model, "vibert-capu.onnx"), "wb").close()
    current["session"] = None
    gec = GecBERTModel(vocab_path=vocab, model_paths=[model], split_chunk=True, chunk_size=56,
                       overlap_size=16, max_len=80, iterations=3, confidence=0.3,
                       case_confidence=0.0)
    rest = object.__new__(ImprovedPunctuationRestorer)
    rest.gec_model = gec
    res = []
    for c in cases():
        sess = Recorder(make_session(c["session"]))
        gec.sessions = [sess]
        with contextlib.redirect_stdout(io.StringIO()):
            if c["kind"] == "restore":
                c["out"] = rest.restore(c["text"], pause_hints=c["pause_hints"])
            else:
                c["out"] = gec([t for t in c["texts"]], pause_hints=c["pause_hints"])
        c["calls"] = sess.calls
        if c["session"]["kind"] == "oracle":
            c["min_margin"] = min(sess.inner.margins)
            sess.inner.margins.clear()
        res.append(c)
        o = c["out"] if isinstance(c["out"], str) else " | ".join(c["out"])
        print(c["kind"], c["session"]["kind"], len(c["calls"]), "runs:", o[:100])
    shutil.rmtree(tmp)
    with open(os.path.join(HERE, "punct_cases.json"), "w", encoding="utf-8") as f:
        json.dump(res, f, ensure_ascii=False, indent=0)
    print("punct_cases.json", len(res), "cases")


if __name__ == "__main__":
    main()
