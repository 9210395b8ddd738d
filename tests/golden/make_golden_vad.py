"""Generate Silero VAD golden fixtures by running the REFERENCE's own vad_utils functions
(build container only; the reference never travels to the GPU box):

    python tests/golden/make_golden_vad.py

The reference's core/vad_utils.py is imported from /root/reference and its lazily created
onnxruntime session (`_vad_session`, :13-38) is set to an object with the same
run(None, {"input", "state", "sr"}) surface that evaluates oracle.silero's restatement of the
silero-vad v5 network on this repo's seeded synthetic weights (the real
silero_vad_16k_op15.onnx is not available offline).  The reference's own code then does
everything else: the 64-sample context, the carried LSTM state, the threshold / min-silence /
min-speech state machine, the low-amplitude boost, the retry at 0.3, the fallback, padding and
merging (core/vad_utils.py:62-260).

Writes tests/golden/vad_golden.json: per case the audio recipe (regenerated bit-identically
by `case_audio`, with a checksum), the call's kwargs, the reference's result and the
probabilities it cached (get_cached_vad_probs, :51-55).
"""
from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
WSEED = 20261019

CASES = [
    # (name, audio recipe, function, kwargs)
    ("speech20", {"kind": "speech", "sec": 20.0, "seed": 31}, "get_vad_segments", {}),
    ("quiet_boost", {"kind": "speech", "sec": 12.0, "seed": 32, "gain": 0.005},
     "get_vad_segments", {}),
    ("boosted_noise", {"kind": "noise", "sec": 6.0, "seed": 33, "gain": 1e-4},
     "get_vad_segments", {}),
    ("silence_fallback", {"kind": "zeros", "sec": 6.0, "seed": 0}, "get_vad_segments", {}),
    ("silence_empty", {"kind": "zeros", "sec": 6.0, "seed": 0}, "get_vad_segments",
     {"fallback_full": False}),
    ("gappy", {"kind": "gappy", "sec": 30.0, "seed": 38}, "get_vad_segments", {}),
    ("gappy_windows", {"kind": "gappy", "sec": 30.0, "seed": 38}, "_run_vad_inference",
     {"threshold": 0.5, "min_silence_ms": 300, "min_speech_ms": 250}),
    ("tiny", {"kind": "speech", "sec": 300 / 16000, "seed": 34}, "get_vad_segments", {}),
    ("burst_retry", {"kind": "burst", "sec": 6.0, "seed": 35, "burst": 0.06},
     "get_vad_segments", {"threshold": 0.5}),
    ("ragged", {"kind": "speech", "sec": 7.3, "seed": 36}, "get_vad_segments",
     {"threshold": 0.5, "padding_ms": 200, "merge_gap_ms": 0}),
    ("windows_default", {"kind": "speech", "sec": 20.0, "seed": 31}, "_run_vad_inference", {}),
    ("windows_strict", {"kind": "speech", "sec": 15.0, "seed": 37}, "_run_vad_inference",
     {"threshold": 0.9, "min_silence_ms": 50, "min_speech_ms": 500}),
]


def case_audio(spec) -> np.ndarray:
    """The case's audio, regenerated from its recipe (zasr.synth_audio is deterministic)."""
    sys.path[:0] = [p for p in (REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd"))
                    if p not in sys.path]
    from zasr.synth_audio import synth_speech
    n = int(round(spec["sec"] * 16000))
    if spec["kind"] == "speech":
        a = synth_speech(max(spec["sec"], 0.5), spec["seed"])[:n]
    elif spec["kind"] == "noise":
        a = np.random.Generator(np.random.PCG64(spec["seed"])).normal(size=n)
    elif spec["kind"] == "zeros":
        a = np.zeros(n)
    elif spec["kind"] == "gappy":  # speech runs separated by 2.5-6 s of digital silence
        rng = np.random.Generator(np.random.PCG64(spec["seed"]))
        sp = synth_speech(spec["sec"], spec["seed"])
        a = np.zeros(n)
        pos = 0
        while pos < n:
            run = int(rng.uniform(1.0, 5.0) * 16000)
            a[pos:pos + run] = sp[pos:pos + run]
            pos += run + int(rng.uniform(2.5, 6.0) * 16000)
    else:  # a short speech burst in the middle of digital silence
        a = np.zeros(n)
        b = synth_speech(1.0, spec["seed"])
        m = int(spec["burst"] * 16000)
        a[n // 2:n // 2 + m] += b[4000:4000 + m] / max(1e-6, float(np.max(np.abs(b[4000:4000 + m])))) * 0.3
    a = np.asarray(a, np.float32) * np.float32(spec.get("gain", 1.0))
    return np.ascontiguousarray(a, np.float32)


def checksum(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, np.float32).tobytes()).hexdigest()[:16]


def main():
    sys.path[:0] = [REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd"), REF]
    import torch
    torch.set_num_threads(4)
    from oracle.silero import SileroOracle
    from zasr.silero import SileroConfig, synth_weights
    with contextlib.redirect_stdout(io.StringIO()):
        import core.vad_utils as ref
    assert os.path.realpath(ref.__file__).startswith(REF), ref.__file__
    cfg = SileroConfig()
    ref._vad_session = SileroOracle(cfg, synth_weights(cfg, WSEED)).session()
    out = {"weights_seed": WSEED, "cases": []}
    for name, spec, fn, kw in CASES:
        a = case_audio(spec)
        ref._last_vad_probs = None
        with contextlib.redirect_stdout(io.StringIO()):
            res = getattr(ref, fn)(a, **kw)
        probs = ref.get_cached_vad_probs()
        out["cases"].append({
            "name": name, "audio": spec, "n_samples": int(a.shape[0]), "sha": checksum(a),
            "fn": fn, "kwargs": kw, "result": [[int(s), int(e)] for s, e in res],
            "probs": None if probs is None else [float(p) for p in probs]})
        print(name, len(a), fn, res[:6], "..." if len(res) > 6 else "",
              None if probs is None else len(probs))
    with open(os.path.join(HERE, "vad_golden.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("vad_golden.json")


if __name__ == "__main__":
    main()
