"""the reference's model directory format, on CPU (host-only loader).

tests/golden/write_onnx.py writes encoder-/decoder-/joiner-*.onnx files from seeded weights in
the torch.onnx export style (linear weights transposed under generated names, MatMul nodes
with scope names, Add bias nodes; int8 variants quantize_dynamic-style).  libzasr's loader
(csrc/onnx_io.cpp, zasr_convert_model) must return exactly the original tensors under the
engine's names, infer the architecture, and pick files like create_recognizer
(core/asr_engine.py:913-928): non-int8 preferred, the int8 file when it is the only one.
The real exported graphs are absent offline: their tensor naming is parity-unpinned."""
import json
import os
import shutil

import numpy as np
import pytest
from safetensors.numpy import load_file

from write_onnx import dequantized, write_model_dir
from zasr.binding import convert_model
from zasr.model import ZipformerConfig, synth_tokens, synth_weights, zipformer_s, zipformer_tiny


def _convert(src, tmp_path, name="out"):
    out = str(tmp_path / name)
    convert_model(src, out)
    with open(os.path.join(out, "config.json")) as f:
        cfg = ZipformerConfig.from_json(f.read())
    return cfg, load_file(os.path.join(out, "model.safetensors"))


def _same_arch(a: ZipformerConfig, b: ZipformerConfig):
    for k in ("encoder_dims", "num_layers", "ff_dims", "num_heads", "downsampling", "cnn_kernels",
              "query_head_dim", "value_head_dim", "pos_head_dim", "pos_dim", "vocab_size",
              "decoder_dim", "joiner_dim", "context_size", "layer1_channels", "layer2_channels",
              "layer3_channels"):
        assert tuple(np.atleast_1d(getattr(a, k))) == tuple(np.atleast_1d(getattr(b, k))), k


@pytest.mark.parametrize("scope_names", [True, False])
def test_float_onnx_dir_loads_bit_exact(tmp_path, scope_names):
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, 11)
    src = str(tmp_path / "model")
    write_model_dir(src, w, synth_tokens(64), scope_names=scope_names)
    got_cfg, got = _convert(src, tmp_path)
    _same_arch(got_cfg, cfg)
    assert set(got) == set(w)
    for k, v in w.items():
        assert got[k].shape == v.shape, k
        np.testing.assert_array_equal(got[k], v, err_msg=k)


def test_30m_shapes_infer_architecture(tmp_path):
    """The real 30M architecture (every stack / downsampling / kernel size inferred)."""
    cfg = zipformer_s()
    w = synth_weights(cfg, 5)
    src = str(tmp_path / "model")
    write_model_dir(src, w, synth_tokens(cfg.vocab_size))
    got_cfg, got = _convert(src, tmp_path)
    _same_arch(got_cfg, cfg)
    for k in ("encoder.encoders.3.encoder.layers.1.feed_forward3.out_proj.weight",
              "encoder.encoders.0.layers.0.self_attn_weights.linear_pos.weight",
              "joiner.output_linear.weight", "decoder.conv.weight", "encoder_proj.weight"):
        np.testing.assert_array_equal(got[k], w[k], err_msg=k)


def test_float_file_preferred_over_int8(tmp_path):
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, 12)
    src = str(tmp_path / "model")
    write_model_dir(src, w, synth_tokens(64), also_int8=True)
    assert any(f.endswith(".int8.onnx") for f in os.listdir(src))
    _, got = _convert(src, tmp_path)
    for k, v in w.items():
        np.testing.assert_array_equal(got[k], v, err_msg=k)


def test_int8_only_dir_is_dequantized(tmp_path):
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, 13)
    src = str(tmp_path / "model")
    write_model_dir(src, w, synth_tokens(64), int8=True)
    _, got = _convert(src, tmp_path)
    want = dequantized(w)
    for k, v in want.items():
        np.testing.assert_array_equal(got[k], v, err_msg=k)
    # the dequantized linear weights really differ from the float ones (int8 was read)
    k = "joiner.output_linear.weight"
    assert not np.array_equal(got[k], w[k])


def test_missing_part_raises_file_not_found(tmp_path):
    cfg = zipformer_tiny(64)
    src = str(tmp_path / "model")
    files = write_model_dir(src, synth_weights(cfg, 14), synth_tokens(64))
    os.remove(files["joiner"])
    with pytest.raises(FileNotFoundError):
        _convert(src, tmp_path)


def test_safetensors_dir_roundtrip(tmp_path):
    """The engine's own format goes through the same loader unchanged."""
    from zasr.model import save_model_dir
    cfg = zipformer_tiny(64)
    w = synth_weights(cfg, 15)
    src = str(tmp_path / "model")
    save_model_dir(src, cfg, w, synth_tokens(64))
    got_cfg, got = _convert(src, tmp_path)
    _same_arch(got_cfg, cfg)
    for k, v in w.items():
        np.testing.assert_array_equal(got[k], v, err_msg=k)


def test_dropin_create_recognizer_accepts_onnx_dir_files(tmp_path):
    """create_recognizer's file check (reference :913-928) accepts the ONNX set and raises
    FileNotFoundError like the reference when tokens.txt is missing (before any GPU use)."""
    import zasr.asr_engine as ae
    cfg = zipformer_tiny(64)
    src = str(tmp_path / "model")
    write_model_dir(src, synth_weights(cfg, 16), synth_tokens(64))
    assert ae.model_files_present(src)
    os.remove(os.path.join(src, "tokens.txt"))
    assert not ae.model_files_present(src)
    with pytest.raises(FileNotFoundError):
        ae.create_recognizer(src)


# ------------------------------------------------------------------ hostile / corrupt files
def _write_enc_with(src, extra_init: bytes):
    """Replace the encoder file of a valid tiny model dir with one whose graph carries one more
    initializer (raw protobuf bytes)."""
    import glob
    from write_onnx import _bytes
    enc = glob.glob(os.path.join(src, "encoder-*.onnx"))[0]
    data = open(enc, "rb").read()
    # append to the graph: ModelProto field 7 is re-emitted with the extra GraphProto.initializer
    from write_onnx import _key, _varint
    graph = _bytes(5, extra_init)
    with open(enc, "wb") as f:
        f.write(data + _key(7, 2) + _varint(len(graph)) + graph)


def _tiny_dir(tmp_path):
    cfg = zipformer_tiny(64)
    src = str(tmp_path / "model")
    write_model_dir(src, synth_weights(cfg, 11), synth_tokens(64))
    return src


def test_truncated_onnx_raises_not_crashes(tmp_path):
    """A truncated file is an error at every cut point class (inside a varint, a length-
    delimited field, a fixed-width field), never a read past the buffer."""
    import glob
    from zasr.binding import ZasrError
    src = _tiny_dir(tmp_path)
    enc = glob.glob(os.path.join(src, "encoder-*.onnx"))[0]
    data = open(enc, "rb").read()
    for cut in (1, 2, 7, 100, len(data) // 3, len(data) - 5, len(data) - 1):
        with open(enc, "wb") as f:
            f.write(data[:cut])
        with pytest.raises(ZasrError):
            convert_model(src, str(tmp_path / f"out{cut}"))


def test_external_data_outside_model_dir_rejected(tmp_path):
    from write_onnx import _bytes, _key, _str, _varint
    from zasr.binding import ZasrError
    for loc in ("../secret.bin", "/etc/passwd", "a/../../b"):
        src = _tiny_dir(tmp_path / loc.replace("/", "_").replace(".", "d"))
        entry = lambda k, v: _bytes(13, _str(1, k) + _str(2, v))  # noqa: E731
        t = (_key(1, 0) + _varint(4) + _key(2, 0) + _varint(1) + _str(8, "encoder.extra")
             + entry("location", loc) + entry("offset", "0") + entry("length", "16")
             + _key(14, 0) + _varint(1))
        _write_enc_with(src, t)
        with pytest.raises(ZasrError, match="external data"):
            convert_model(src, str(tmp_path / "o" / loc.replace("/", "_")))


def test_negative_dims_rejected(tmp_path):
    from write_onnx import _bytes, _key, _str, _varint
    from zasr.binding import ZasrError
    src = _tiny_dir(tmp_path)
    neg = _varint((1 << 64) - 3)  # int64 -3 as a protobuf varint
    t = _key(1, 0) + neg + _key(2, 0) + _varint(1) + _str(8, "encoder.bad") + _bytes(9, b"")
    _write_enc_with(src, t)
    with pytest.raises(ZasrError, match="negative"):
        convert_model(src, str(tmp_path / "out"))
