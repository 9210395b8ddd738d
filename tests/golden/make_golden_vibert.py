"""Generate ViBERT golden fixtures by running the REFERENCE's own model class (build container
only):

    python tests/golden/make_golden_vibert.py

The reference's convert_onnx/export_vibert_onnx.py Seq2LabelsModel (the module it exports to
vibert-capu.onnx) is built offline from a local BertConfig (the config the reference reads via
AutoConfig.from_pretrained(pretrained_name_or_path), written from zasr.vibert.VibertConfig),
loaded with this repo's seeded synthetic weights, eval mode, and run on seeded inputs laid out
like GecBERTModel.preprocess makes them (core/gec_model.py:447-480: START token first, padded
batch, attention mask, zero token types, word-start offsets padded with 0).

Writes tests/golden/vibert_golden.npz: per case the config name, weight seed, inputs and the
reference's (logits, detect_logits).
"""
from __future__ import annotations

import contextlib
import importlib.util
import io
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd")]


def make_inputs(cfg, B, max_words, seed):
    """A padded batch the way GecBERTModel.preprocess builds it: START token (the last id)
    first, 1-3 sub-tokens per word, offsets = first sub-token of each word (0 = START)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    seqs, offs = [], []
    for b in range(B):
        nw = int(rng.integers(max(1, max_words // 3), max_words + 1))
        toks, o = [cfg.vocab_size - 1], [0]
        for _ in range(nw):
            o.append(len(toks))
            toks += [int(t) for t in rng.integers(1, cfg.vocab_size - 1, size=int(rng.integers(1, 4)))]
        seqs.append(toks)
        offs.append(o)
    L = max(len(s) for s in seqs)
    W = max(len(o) for o in offs)
    ids = np.zeros((B, L), np.int64)
    am = np.zeros((B, L), np.int64)
    off = np.zeros((B, W), np.int64)
    for b, (s, o) in enumerate(zip(seqs, offs)):
        ids[b, :len(s)] = s
        am[b, :len(s)] = 1
        off[b, :len(o)] = o
    return ids, am, np.zeros_like(ids), off


def main():
    import torch
    from zasr.vibert import synth_weights, vibert_base, vibert_tiny
    torch.set_num_threads(8)
    spec = importlib.util.spec_from_file_location(
        "ref_export_vibert", os.path.join(REF, "convert_onnx", "export_vibert_onnx.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    out = {}
    cases = [("tiny", vibert_tiny(), 11, 4, 12, 501), ("tiny", vibert_tiny(), 11, 32, 40, 502),
             ("base", vibert_base(), 12, 3, 16, 503)]
    for ci, (kind, cfg, wseed, B, maxw, iseed) in enumerate(cases):
        d = tempfile.mkdtemp()
        with open(os.path.join(d, "config.json"), "w") as f:
            json.dump(cfg.bert_config_json(), f)
        rcfg = ref.Seq2LabelsConfig(pretrained_name_or_path=d, vocab_size=cfg.num_labels,
                                    num_detect_classes=cfg.num_detect_classes,
                                    load_pretrained=False, special_tokens_fix=True,
                                    num_labels=cfg.num_labels)
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            net = ref.Seq2LabelsModel(rcfg).eval()
        w = synth_weights(cfg, wseed)
        net.load_state_dict({k: torch.from_numpy(v) for k, v in w.items()}, strict=True)
        ids, am, tt, off = make_inputs(cfg, B, maxw, iseed)
        with torch.no_grad():
            lg, dl = net(input_ids=torch.from_numpy(ids), attention_mask=torch.from_numpy(am),
                         token_type_ids=torch.from_numpy(tt), input_offsets=torch.from_numpy(off),
                         return_dict=False)[:2]
        p = f"c{ci}_"
        out[p + "kind"] = np.array(kind)
        out[p + "wseed"] = np.array(wseed)
        for k, v in (("input_ids", ids), ("attention_mask", am), ("token_type_ids", tt),
                     ("input_offsets", off)):
            out[p + k] = v
        out[p + "logits"] = lg.numpy().astype(np.float32)
        out[p + "detect_logits"] = dl.numpy().astype(np.float32)
        print(kind, ids.shape, off.shape, "->", tuple(lg.shape), tuple(dl.shape))
    np.savez_compressed(os.path.join(HERE, "vibert_golden.npz"), **out)
    print("vibert_golden.npz")


if __name__ == "__main__":
    main()
