"""Development tool: decode the bench hour once with beam 8 + hotword.txt through a libzasr
built with -DZASR_SEARCH_STAMPS (tools/ab_variant.sh ssstamp search_kernels.hip
"-DZASR_SEARCH_STAMPS"); search_step_kernel's block 0 prints its mean per-phase shader cycles
at the last frame.  usage: ZASR_LIB=ablib/ssstamp/libzasr.so python tools/search_stamps.py [prec]"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from zasr.binding import Recognizer  # noqa: E402
from zasr.model import PRESETS, save_model_dir, synth_tokens, variant_weights  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
cfg = PRESETS["zipformer-68m"]()
mdir = os.path.join(tempfile.gettempdir(), f"zasr_stamps_{os.getpid()}")
save_model_dir(mdir, cfg, variant_weights(cfg, bench.WEIGHT_SEED, "greedy-calibrated"),
               synth_tokens(cfg.vocab_size))
hw = bench.load_hotwords(bench.DEFAULT_HOTWORDS, cfg.vocab_size)
chunks = bench.make_chunks(3600.0, bench.AUDIO_SEED)
lens = [c.shape[0] for c in chunks]
offs = np.cumsum([0] + lens[:-1]).tolist()
d = torch.from_numpy(np.concatenate(chunks)).cuda()
rec = Recognizer(mdir, "modified_beam_search", 8, hotwords=hw[0], hotword_scores=hw[1],
                 precision=prec)
for _ in range(2):
    rec.decode_device(d.data_ptr(), offs, lens, beam=8)
    torch.cuda.synchronize()
rec.close()
print("ok", flush=True)
