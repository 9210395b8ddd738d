"""Write a synthetic reference-style model directory (encoder-/decoder-/joiner-*.onnx +
tokens.txt) from seeded Zipformer weights, for the ONNX initializer loader tests.

The files follow what torch.onnx / icefall's export-onnx.py produce for the three graphs the
reference opens with onnxruntime (core/asr_engine.py:913-928): conv / embedding / norm /
bias tensors keep their module names; every nn.Linear weight is stored TRANSPOSED ([in][out])
under a generated "onnx::MatMul_<n>" name and consumed by a MatMul node whose name is the
module scope ("/encoder/encoders.0/layers.0/feed_forward1/in_proj/MatMul"), followed by an Add
with the named bias.  `scope_names=False` drops the node names (the loader then names a weight
from the Add's bias), and `int8=True` writes onnxruntime quantize_dynamic-style weights
("<w>_quantized" int8 + "<w>_scale" + "<w>_zero_point", MatMulInteger).  The encoder also
carries one positional-encoding constant per stack ("onnx::Slice_<n>", 1999 x 48 f32), as the
traced icefall graph does (tests/test_encoder_bytes.py), which the loader must pass over.

Only the initializers (and the nodes that name them) matter to this build: it does not run the
graphs.  Protobuf wire format is written by hand (the onnx package is not installed).
"""
from __future__ import annotations

import os
from typing import Dict, List, Tuple

import numpy as np

FLOAT, UINT8, INT8 = 1, 2, 3


def _varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _bytes(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _str(field: int, s: str) -> bytes:
    return _bytes(field, s.encode("utf-8"))


def tensor_proto(name: str, arr: np.ndarray, dtype: int) -> bytes:
    out = b"".join(_key(1, 0) + _varint(int(d)) for d in arr.shape)  # dims, unpacked
    out += _key(2, 0) + _varint(dtype)
    out += _str(8, name)
    np_t = {FLOAT: "<f4", UINT8: "u1", INT8: "i1"}[dtype]
    out += _bytes(9, np.ascontiguousarray(arr, dtype=np_t).tobytes())
    return out


def node_proto(op: str, inputs: List[str], outputs: List[str], name: str = "") -> bytes:
    out = b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outputs)
    if name:
        out += _str(3, name)
    return out + _str(4, op)


def model_proto(nodes: List[bytes], inits: List[bytes]) -> bytes:
    graph = b"".join(_bytes(1, n) for n in nodes) + _str(2, "main_graph") + \
        b"".join(_bytes(5, t) for t in inits)
    return _key(1, 0) + _varint(8) + _bytes(7, graph) + \
        _bytes(8, _str(1, "") + _key(2, 0) + _varint(17))  # ir_version, graph, opset 17


def is_linear_weight(name: str, w: Dict[str, np.ndarray]) -> bool:
    if not name.endswith(".weight") or w[name].ndim != 2:
        return False
    return not name.startswith(("decoder.embedding", "encoder_embed.convnext"))


def quantize(a: np.ndarray) -> Tuple[np.ndarray, np.float32, np.int8]:
    scale = np.float32(max(float(np.abs(a).max()), 1e-8) / 127.0)
    q = np.clip(np.rint(a / scale), -127, 127).astype(np.int8)
    return q, scale, np.int8(0)


def graph_for(names: List[str], w: Dict[str, np.ndarray], strip: str, scope_names: bool,
              int8: bool, counter: List[int]):
    nodes, inits = [], []
    for name in names:
        a = w[name]
        local = name[len(strip):] if strip and name.startswith(strip) else name
        if is_linear_weight(name, w):
            counter[0] += 1
            gen = f"onnx::MatMul_{counter[0]}"
            mod = local[: -len(".weight")]
            scope = "/" + mod.replace(".", "/") + "/MatMul" if scope_names else ""
            out = f"{gen}_out"
            wt = np.ascontiguousarray(a.T)
            if int8:
                q, sc, zp = quantize(wt)
                inits.append(tensor_proto(gen + "_quantized", q, INT8))
                inits.append(tensor_proto(gen + "_scale", np.array(sc, np.float32), FLOAT))
                inits.append(tensor_proto(gen + "_zero_point", np.array(zp, np.int8), INT8))
                nodes.append(node_proto("MatMulInteger", ["x_q", gen + "_quantized", "x_zp",
                                                          gen + "_zero_point"], [out], scope))
                nodes.append(node_proto("Cast", [out], [out + "_f"]))
                nodes.append(node_proto("Mul", [out + "_f", "x_scale"], [out + "_m"]))
                tail = out + "_m"
            else:
                inits.append(tensor_proto(gen, wt, FLOAT))
                nodes.append(node_proto("MatMul", ["x", gen], [out], scope))
                tail = out
            bias = mod + ".bias"
            if strip + bias in names:
                nodes.append(node_proto("Add", [tail, bias], [tail + "_b"]))
        else:
            inits.append(tensor_proto(local, a, FLOAT))
    return nodes, inits


def pe_constants(w: Dict[str, np.ndarray], counter: List[int]):
    """The traced CompactRelPositionalEncoding tables the real encoder graph carries (one per
    encoder stack, (2 * 1000 - 1) x pos_dim f32, computed at construction and held as a plain
    tensor attribute, so the trace bakes each into a generated-name constant sliced by the
    sequence length; tests/test_encoder_bytes.py): the loader must pass over them."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from oracle.zipformer import compact_rel_pos_emb
    stacks = sorted({int(n.split(".")[2]) for n in w if n.startswith("encoder.encoders.")})
    pos_dim = next(a.shape[1] for n, a in w.items() if n.endswith("linear_pos.weight"))
    table = compact_rel_pos_emb(1000, pos_dim).numpy()
    nodes, inits = [], []
    for i in stacks:
        counter[0] += 1
        name = f"onnx::Slice_{counter[0]}"
        inits.append(tensor_proto(name, table, FLOAT))
        nodes.append(node_proto("Slice", [name, "pe_start", "pe_end"], [name + "_out"],
                                f"/encoder/encoders.{i}/encoder_pos/Slice"))
    return nodes, inits


def write_model_dir(path: str, w: Dict[str, np.ndarray], tokens: List[str], tag: str = "epoch-99-avg-1",
                    scope_names: bool = True, int8: bool = False, also_int8: bool = False,
                    pe_tables: bool = True) -> Dict[str, str]:
    """Writes encoder-<tag>.onnx, decoder-<tag>.onnx, joiner-<tag>.onnx (or *.int8.onnx) and
    tokens.txt.  also_int8 additionally writes the int8 variants next to the float files (the
    loader must prefer the float ones); pe_tables adds the encoder's positional-encoding
    constants (pe_constants).  Returns {part: file path}."""
    os.makedirs(path, exist_ok=True)
    parts = {
        "encoder": sorted(n for n in w if n.startswith(("encoder.", "encoder_embed.", "encoder_proj."))),
        "decoder": sorted(n for n in w if n.startswith(("decoder.", "decoder_proj."))),
        "joiner": sorted(n for n in w if n.startswith("joiner.")),
    }
    written = {}
    variants = [int8] if not also_int8 else [False, True]
    for q in variants:
        counter = [100]
        for part, names in parts.items():
            strip = "joiner." if part == "joiner" else ""
            nodes, inits = graph_for(names, w, strip, scope_names, q, counter)
            if part == "encoder" and pe_tables:
                n_, i_ = pe_constants(w, counter)
                nodes, inits = nodes + n_, inits + i_
            fn = os.path.join(path, f"{part}-{tag}{'.int8' if q else ''}.onnx")
            with open(fn, "wb") as f:
                f.write(model_proto(nodes, inits))
            written[part + ("_int8" if q else "")] = fn
    with open(os.path.join(path, "tokens.txt"), "w", encoding="utf-8") as f:
        for i, t in enumerate(tokens):
            f.write(f"{t} {i}\n")
    return written


def dequantized(w: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """The weights an int8 directory holds after dequantization (what the loader must return)."""
    out = {}
    for n, a in w.items():
        if is_linear_weight(n, w):
            q, sc, zp = quantize(np.ascontiguousarray(a.T))
            out[n] = np.ascontiguousarray(((q.astype(np.float32) - np.float32(zp)) * sc).T)
        else:
            out[n] = a
    return out


if __name__ == "__main__":  # pragma: no cover
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__)))), "sherpa-vietnamese-asr_amd"))
    from zasr.model import synth_tokens, synth_weights, zipformer_tiny
    cfg = zipformer_tiny(64)
    print(write_model_dir(sys.argv[1], synth_weights(cfg, 3), synth_tokens(64)))
