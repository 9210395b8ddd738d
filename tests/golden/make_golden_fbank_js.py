"""Fixtures from the reference's OWN executable fbank (test infrastructure only).

The reference ships a second, executable fbank besides its kaldi-native-fbank call
(`core/asr_engine.py:698-721`, knf absent here): `computeFbank` in
`offline_pwa/static/js/pure-ort-asr-worker.js:470-519`.  This script runs that function under
node (`tests/golden/run_reference_fbank.js`, which cuts the fbank's constants and functions out
of the worker file's text and evaluates only those, in a bare vm context, in a child process
with an empty environment)
on seeded inputs and commits its outputs to `tests/golden/fbank_js.npz`:

  lengths 1, 399, 400, 401, 1599, 16000*7 + 123 and 480000 samples of seeded synthetic speech
  (zasr.synth_audio.synth_speech, seed 4242), plus 1600 zeros (the log floor) and a 1 kHz tone.

tests/test_fbank_oracle.py regenerates the same inputs and checks `oracle.fbank.fbank_js`
(the oracle's Hz-triangle mode) against these outputs within 1e-5, and the oracle's kaldi
(mel-triangle) mode against them within the one documented difference (triangle shape).
Run in the build container (needs /root/reference and node):
    python tests/golden/make_golden_fbank_js.py
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "sherpa-vietnamese-asr_amd"))
WORKER = "/root/reference/offline_pwa/static/js/pure-ort-asr-worker.js"
OUT = os.path.join(HERE, "fbank_js.npz")

SPEECH_LENGTHS = [1, 399, 400, 401, 1599, 16000 * 7 + 123, 480000]


def fbank_js_inputs():
    """[(name, float32 samples)] -- the inputs the fixture was made from (deterministic)."""
    from zasr.synth_audio import synth_speech
    speech = synth_speech(30.0, 4242).astype(np.float32)
    assert speech.shape[0] >= max(SPEECH_LENGTHS)
    out = [(f"speech_{n}", speech[:n].copy()) for n in SPEECH_LENGTHS]
    out.append(("zeros_1600", np.zeros(1600, np.float32)))
    t = np.arange(16000, dtype=np.float64) / 16000.0
    out.append(("tone_1k", (0.25 * np.sin(2 * np.pi * 1000.0 * t)).astype(np.float32)))
    return out


def main():
    ins = fbank_js_inputs()
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.f32"), os.path.join(td, "out.f32")
        np.concatenate([x for _, x in ins]).astype(np.float32).tofile(fin)
        lens = ",".join(str(x.shape[0]) for _, x in ins)
        r = subprocess.run(["node", os.path.join(HERE, "run_reference_fbank.js"), WORKER, fin,
                            lens, fout], capture_output=True, text=True, check=True, cwd=td,
                           env={"PATH": "/usr/bin:/bin"}, timeout=600)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        flat = np.fromfile(fout, dtype=np.float32)
    arrays, off = {}, 0
    for name, x in ins:
        T = (x.shape[0] + 80) // 160
        arrays[name] = flat[off:off + T * 80].reshape(T, 80)
        off += T * 80
    assert off == flat.shape[0], (off, flat.shape)
    node = subprocess.run(["node", "--version"], capture_output=True, text=True).stdout.strip()
    meta = {"generator": "tests/golden/make_golden_fbank_js.py + run_reference_fbank.js",
            "reference": "offline_pwa/static/js/pure-ort-asr-worker.js:470-519 computeFbank",
            "node": node, "extracted_functions": info["functions"],
            "names": [n for n, _ in ins]}
    np.savez_compressed(OUT, meta=np.array(json.dumps(meta)), **arrays)
    print(f"wrote {OUT}: {len(ins)} inputs, {off // 80} frames; {meta}")


if __name__ == "__main__":
    main()
