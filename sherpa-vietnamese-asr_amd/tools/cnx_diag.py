"""Development diagnostic: encoder_out of the M-set chunks (tests/test_gpu_e2e.py M_SECS) in
f16x3 with the ConvNeXt MLP on convnext_mlp_h3_kernel (ZASR_CNX_FFN=0) and on the fused f16x3
FFN (default), in several batch orders, against the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from model_fixtures import m_model  # noqa: E402
from oracle.fbank import fbank  # noqa: E402
from oracle.zipformer import ZipformerOracle  # noqa: E402
from test_gpu_e2e import M_SECS, _speech  # noqa: E402
from zasr.binding import Recognizer  # noqa: E402

cfg, w, path = m_model()
orc = ZipformerOracle(cfg, w)
chunks = [_speech(s, 1200 + i) for i, s in enumerate(M_SECS)]
feats = [fbank(c) for c in chunks]
ref = [orc.encoder(f) for f in feats]
print("frames", [f.shape[0] for f in feats])
for env in ("0", "1"):
    os.environ["ZASR_CNX_FFN"] = env
    rec = Recognizer(path, "greedy_search", 1, precision="f16x3")
    for order in ([0, 1, 2], [2, 1, 0], [2], [1], [0, 2], [2, 0]):
        got = rec.encode_features([feats[i] for i in order])
        errs = ["%d:%.1e" % (i, np.max(np.abs(g - ref[i]))) for i, g in zip(order, got)]
        print("ZASR_CNX_FFN=%s order %s -> %s" % (env, order, " ".join(errs)))
    rec.close()
