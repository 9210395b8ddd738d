"""The reader of the reference's single-graph stage models (onnx_io.cpp load_stage_onnx, C-ABI
zasr_convert_stage_model; host only, no GPU): synthetic files in the layouts of
silero_vad_16k_op15.onnx, campplus_cn_en_common_200k.onnx and vibert-capu.onnx(.int8)
(tests/golden/write_stage_onnx.py) load to exactly the seeded weights -- bit for bit, the
LSTM gates back in torch order, a BatchNorm the exporter fused into its Conv as the folded
weight plus "<bn>.fused_shift" -- and to the model's configuration."""
import json
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))

from write_stage_onnx import write_campp, write_silero, write_vibert  # noqa: E402


def _load(out_dir, kind):
    from safetensors.numpy import load_file
    st = {"silero": "silero_vad.safetensors", "campp": "campp.safetensors",
          "vibert": "vibert.safetensors"}[kind]
    w = load_file(os.path.join(out_dir, st))
    cfg = json.load(open(os.path.join(out_dir, f"{kind}_config.json")))
    return w, cfg


def _convert(kind, src, dst):
    from zasr.binding import convert_stage_model
    convert_stage_model(kind, str(src), str(dst))
    return _load(str(dst), kind)


def _same(got, want):
    assert sorted(got) == sorted(want)
    for k in want:
        assert got[k].shape == tuple(want[k].shape), k
        assert np.array_equal(got[k], np.asarray(want[k], np.float32)), k


@pytest.mark.parametrize("variant", ["flat", "if"])
def test_silero_onnx_loads_seeded_weights(tmp_path, variant):
    from zasr.silero import SileroConfig, synth_weights
    cfg = SileroConfig()
    w = synth_weights(cfg, 31)
    write_silero(str(tmp_path / "m"), w, variant)
    got, c = _convert("silero", tmp_path / "m", tmp_path / "o")
    _same(got, w)
    assert SileroConfig.from_json(json.dumps(c)) == cfg


def test_silero_fallback_name_and_missing(tmp_path):
    from zasr.binding import convert_stage_model
    from zasr.silero import SileroConfig, synth_weights
    w = synth_weights(SileroConfig(), 32)
    write_silero(str(tmp_path / "m"), w, "flat", name="silero_vad.onnx")
    got, _ = _convert("silero", tmp_path / "m", tmp_path / "o")
    _same(got, w)
    with pytest.raises(FileNotFoundError):
        convert_stage_model("silero", str(tmp_path / "nothing"), str(tmp_path / "o2"))


@pytest.mark.parametrize("fused", [True, False], ids=["conv_bn_fused", "unfused"])
def test_campp_onnx_loads_seeded_weights(tmp_path, fused):
    from zasr.campp import CamppConfig, synth_weights
    cfg = CamppConfig()
    w = synth_weights(cfg, 33)
    _, want = write_campp(str(tmp_path / "m"), w, fused=fused)
    got, c = _convert("campp", tmp_path / "m", tmp_path / "o")
    _same(got, want)
    if fused:
        # head conv1 / conv2, 2 x 2 res blocks x (conv1, conv2), 2 shortcuts, tdnn, linear1s
        assert sum(k.endswith(".fused_shift") for k in got) == 2 + 8 + 2 + 1 + sum(cfg.block_layers)
    c.setdefault("seg_len", cfg.seg_len)
    assert CamppConfig.from_json(json.dumps(c)) == cfg


@pytest.mark.parametrize("int8", [False, True], ids=["fp32", "int8"])
def test_vibert_onnx_loads_seeded_weights(tmp_path, int8):
    from zasr.vibert import VibertConfig, synth_weights, vibert_tiny
    cfg = vibert_tiny()
    w = synth_weights(cfg, 34)
    _, want = write_vibert(str(tmp_path / "m"), w, int8=int8)
    with open(tmp_path / "m" / "config.json", "w") as f:
        json.dump({"num_attention_heads": cfg.num_attention_heads, "layer_norm_eps": 1e-12,
                   "pretrained_name_or_path": "FPTAI/vibert-base-cased"}, f)
    got, c = _convert("vibert", tmp_path / "m", tmp_path / "o")
    _same(got, want)
    assert VibertConfig(**c) == cfg


def test_vibert_prefers_fp32_and_defaults_head_dim_64(tmp_path):
    from zasr.vibert import VibertConfig, synth_weights
    cfg = VibertConfig(hidden_size=128, num_hidden_layers=1, num_attention_heads=2,
                       intermediate_size=64, vocab_size=50)
    w = synth_weights(cfg, 35)
    _, want = write_vibert(str(tmp_path / "m"), w, int8=False)
    write_vibert(str(tmp_path / "m"), {k: v * 2 for k, v in w.items()}, int8=True)
    got, c = _convert("vibert", tmp_path / "m", tmp_path / "o")
    _same(got, want)                       # vibert-capu.onnx, not the int8 file
    assert c["num_attention_heads"] == 2   # no config.json: hidden / 64
