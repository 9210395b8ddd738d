"""GPU diagnostic (test infrastructure): encoder_out of each precision mode vs the fp32 oracle
on tests/test_gpu_e2e.py's three 68M chunks -- max |diff|, max scaled diff, and the diff of
each mode against the fp32 HIP mode.  Writes gpurun_out/diag_precision.json."""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "sherpa-vietnamese-asr_amd")]


def main(modes):
    from model_fixtures import m_model
    from oracle.fbank import fbank
    from oracle.zipformer import ZipformerOracle
    from test_gpu_e2e import M_SECS, _speech
    from zasr.binding import Recognizer
    cfg, w, path = m_model()
    orc = ZipformerOracle(cfg, w)
    feats = [fbank(_speech(s, 1200 + i)) for i, s in enumerate(M_SECS)]
    refs = [orc.encoder(f) for f in feats]
    out, got = {}, {}
    for m in modes:
        rec = Recognizer(path, "greedy_search", 1, precision=m)
        got[m] = rec.encode_features(feats)
        rec.close()
        out[m] = {"max_abs_vs_oracle": [float(np.abs(g - r).max()) for g, r in zip(got[m], refs)],
                  "rms_vs_oracle": [float(np.sqrt(np.mean((g - r) ** 2))) for g, r in zip(got[m], refs)]}
        if "fp32" in got and m != "fp32":
            out[m]["max_abs_vs_fp32"] = [float(np.abs(g - r).max()) for g, r in zip(got[m], got["fp32"])]
        print(m, json.dumps(out[m]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/diag_precision.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:] or ["fp32", "bf16x6", "bf16x3", "bf16"])
