"""Generate CAM++ golden fixtures by running the REFERENCE's own Python (build container only).

    python tests/golden/make_golden_campp.py

* Embeddings: the reference's CAMPPlus class (convert_onnx/export_campplus_onnx.py:17-270,
  the exact module the reference exported to ONNX) built with the exporter's configuration,
  loaded with this repo's seeded synthetic weights (zasr.campp.synth_weights, incl. random BN
  running statistics), eval mode, run on seeded feature batches -- random (N, T, 80) batches
  and a batch laid out like the reference pipeline (fbank windows of synthetic speech, 150
  frames, zero-padded to the batch maximum, core/speaker_diarization_senko_campp_optimized.py:
  589-605).
* fbank: the reference's _compute_fbank_vectorized (:86-159) on seeded audio.  Its mel matrix
  normally comes from kaldi_native_fbank, which is absent: the module global is set to
  oracle.campplus.kaldi_mel_bank() (the matrix is therefore not pinned; everything else --
  scaling, framing, pre-emphasis, window, FFT, floor, log, CMVN -- is the reference's code).

Writes tests/golden/campp_golden.npz (inputs, outputs and the weight seed).
"""
from __future__ import annotations

import contextlib
import importlib.util
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [REPO, os.path.join(REPO, "sherpa-vietnamese-asr_amd")]

WEIGHT_SEED = 4242


def _ref_campp_module():
    spec = importlib.util.spec_from_file_location(
        "ref_export_campplus", os.path.join(REF, "convert_onnx", "export_campplus_onnx.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _ref_fbank_fn():
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        import core.speaker_diarization_senko_campp_optimized as sd
    from oracle.campplus import kaldi_mel_bank
    sd._fbank_mel_bank = kaldi_mel_bank()
    hann = 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(400) / 399)
    sd._fbank_povey_window = np.power(hann, 0.85).astype(np.float32)
    return sd._compute_fbank_vectorized


def pipeline_batch(fbank_fn, seed: int):
    """Windows of two speech regions (one shorter than a window) as the reference batches them."""
    from zasr.campp import window_plan
    from zasr.synth_audio import synth_speech
    regions = [synth_speech(4.3, seed), synth_speech(1.1, seed + 1)]
    slices = []
    for a in regions:
        fb = fbank_fn(a)
        for s, n in window_plan(fb.shape[0]):
            slices.append(fb[s:s + n])
    T = max(s.shape[0] for s in slices)
    batch = np.zeros((len(slices), T, 80), np.float32)
    for i, s in enumerate(slices):
        batch[i, :s.shape[0]] = s
    return batch


def main():
    import torch
    from zasr.campp import CamppConfig, synth_weights
    from zasr.synth_audio import synth_speech
    torch.set_num_threads(8)
    ref = _ref_campp_module()
    fbank_fn = _ref_fbank_fn()
    cfg = CamppConfig()
    net = ref.CAMPPlus(feat_dim=80, embedding_size=192, growth_rate=32, bn_size=4,
                       init_channels=128, config_str="batchnorm-relu", memory_efficient=True)
    w = synth_weights(cfg, WEIGHT_SEED)
    sd = {k: torch.from_numpy(v) for k, v in w.items()}
    for k, v in net.state_dict().items():
        if k.endswith("num_batches_tracked"):
            sd[k] = v
    net.load_state_dict(sd, strict=True)
    net.eval()
    out = {"weight_seed": np.array(WEIGHT_SEED)}
    rng = np.random.Generator(np.random.PCG64(77))
    cases = {"rand_3x150": rng.normal(0, 1, (3, 150, 80)).astype(np.float32),
             "rand_2x97": rng.normal(0, 1, (2, 97, 80)).astype(np.float32),
             "rand_1x230": rng.normal(0, 1, (1, 230, 80)).astype(np.float32),
             "pipeline": pipeline_batch(fbank_fn, 900)}
    with torch.no_grad():
        for name, x in cases.items():
            out[f"emb_in_{name}"] = x
            out[f"emb_out_{name}"] = net(torch.from_numpy(x)).numpy().astype(np.float32)
            print(name, x.shape, "->", out[f"emb_out_{name}"].shape)
    for i, sec in enumerate((1.7, 3.0, 0.0251, 0.0249)):
        a = synth_speech(max(sec, 0.01), 910 + i)[: int(round(sec * 16000))]
        out[f"fb_in_{i}"] = a.astype(np.float32)
        out[f"fb_out_{i}"] = fbank_fn(a)
        print("fbank", a.shape, "->", out[f"fb_out_{i}"].shape)
    np.savez_compressed(os.path.join(HERE, "campp_golden.npz"), **out)
    print("campp_golden.npz")


if __name__ == "__main__":
    main()
