"""Write synthetic reference-layout ONNX files of the three single-graph stage models from
seeded weights, for the stage-model reader tests (onnx_io.cpp load_stage_onnx).

The layouts follow what produced the files the reference opens:
* silero_vad_16k_op15.onnx (core/vad_utils.py:22-24; snakers4/silero-vad, third-party): the
  16 kHz network as ONNX ops -- Pad, STFT Conv with the basis buffer, magnitude, four kernel-3
  encoder Convs (strides / pads attributes), an LSTM node whose W / R / B are torch's
  LSTMCell parameters in ONNX gate order (i, o, f, c) under generated names, Relu, the
  [1][128][1] output Conv, Sigmoid.  variant "if": the graph silero ships for both rates --
  an If node whose then-branch is the 8 kHz network (basis [130][1][128]) and whose
  else-branch is the 16 kHz one, the initializers inside the branches and the 16 kHz basis
  as a Constant node.
* campplus_cn_en_common_200k.onnx (convert_onnx/export_campplus_onnx.py:346-359: torch.onnx,
  opset 17, do_constant_folding, eval): Conv / BatchNormalization nodes named by scope path.
  fused=True: every Conv directly followed by its BatchNorm carries the folded weight
  W * gamma / sqrt(var + eps) and bias beta - mean * gamma / sqrt(var + eps) under generated
  names, as the exporter's eval-mode Conv+BN fusion leaves it; the BatchNorms after ReLU or
  Squeeze stay BatchNormalization nodes with their named parameters.
* vibert-capu.onnx (convert_onnx/export_vibert_onnx.py:283-304: the model inside the
  _ViBERTForExport wrapper, so every name starts with "model."): embeddings / LayerNorm /
  biases named, every nn.Linear weight transposed under "onnx::MatMul_<n>" with a scoped
  MatMul node ("/model/bert/encoder/layer.0/attention/self/query/MatMul") and an Add of the
  named bias; int8=True: onnxruntime quantize_dynamic's MatMulInteger layout.

Only initializers, node inputs, node names and the attributes the reader uses matter; the
graphs are not meant to run.  Protobuf wire format by hand (write_onnx.py helpers).
"""
from __future__ import annotations

import os
from typing import Dict, List

import numpy as np

from write_onnx import (FLOAT, INT8, _bytes, _key, _str, _varint, model_proto, node_proto,
                        quantize, tensor_proto)

BN_EPS = 1e-5


def attr_ints(name: str, vals: List[int]) -> bytes:
    out = _str(1, name) + _key(20, 0) + _varint(7)  # type INTS
    return out + b"".join(_key(8, 0) + _varint(int(v) & ((1 << 64) - 1)) for v in vals)


def attr_int(name: str, v: int) -> bytes:
    return _str(1, name) + _key(20, 0) + _varint(2) + _key(3, 0) + _varint(int(v))


def attr_graph(name: str, graph: bytes) -> bytes:
    return _str(1, name) + _key(20, 0) + _varint(5) + _bytes(6, graph)


def attr_tensor(name: str, t: bytes) -> bytes:
    return _str(1, name) + _key(20, 0) + _varint(4) + _bytes(5, t)


def node(op: str, inputs: List[str], outputs: List[str], name: str = "", attrs=()) -> bytes:
    return node_proto(op, inputs, outputs, name) + b"".join(_bytes(5, a) for a in attrs)


def graph_proto(nodes: List[bytes], inits: List[bytes], name: str = "g") -> bytes:
    return b"".join(_bytes(1, n) for n in nodes) + _str(2, name) + b"".join(_bytes(5, t) for t in inits)


def write_model(path: str, nodes: List[bytes], inits: List[bytes]) -> str:
    with open(path, "wb") as f:
        f.write(model_proto(nodes, inits))
    return path


# ------------------------------------------------------------------------------ Silero
def onnx_gates(a: np.ndarray, H: int) -> np.ndarray:
    """torch LSTMCell gate blocks (i, f, g, o) -> ONNX LSTM (i, o, f, c)."""
    i, f, g, o = (a[k * H:(k + 1) * H] for k in range(4))
    return np.concatenate([i, o, f, g], 0)


def silero_graph(w: Dict[str, np.ndarray], tag: str, basis_const: bool, counter: List[int],
                 strides=(1, 2, 2, 1)):
    P = "_model."
    nodes, inits = [], []
    basis = w[P + "stft.forward_basis_buffer"]
    fl = basis.shape[2]
    nodes.append(node("Pad", ["x", "pads"], [f"{tag}pad"], f"/{tag}stft/padding/Pad"))
    bname = P + "stft.forward_basis_buffer"
    if basis_const:
        counter[0] += 1
        bname = f"onnx::Conv_{counter[0]}"
        nodes.append(node("Constant", [], [bname], f"/{tag}stft/Constant",
                          [attr_tensor("value", tensor_proto("", basis, FLOAT))]))
    else:
        inits.append(tensor_proto(bname, basis, FLOAT))
    nodes.append(node("Conv", [f"{tag}pad", bname], [f"{tag}spec"], f"/{tag}stft/Conv",
                      [attr_ints("strides", [fl // 2]), attr_ints("kernel_shape", [fl])]))
    nodes.append(node("Sqrt", [f"{tag}spec"], [f"{tag}mag"], f"/{tag}stft/Sqrt"))
    cur = f"{tag}mag"
    i = 0
    while P + f"encoder.{i}.reparam_conv.weight" in w:
        cw, cb = w[P + f"encoder.{i}.reparam_conv.weight"], w[P + f"encoder.{i}.reparam_conv.bias"]
        stride = strides[i]
        wn, bn = P + f"encoder.{i}.reparam_conv.weight", P + f"encoder.{i}.reparam_conv.bias"
        if tag:
            wn, bn = tag + wn, tag + bn
        inits += [tensor_proto(wn, cw, FLOAT), tensor_proto(bn, cb, FLOAT)]
        nodes.append(node("Conv", [cur, wn, bn], [f"{tag}e{i}"], f"/{tag}encoder/{i}/reparam_conv/Conv",
                          [attr_ints("strides", [int(stride)]), attr_ints("pads", [1, 1]),
                           attr_ints("kernel_shape", [3])]))
        nodes.append(node("Relu", [f"{tag}e{i}"], [f"{tag}r{i}"], f"/{tag}encoder/{i}/activation/Relu"))
        cur = f"{tag}r{i}"
        i += 1
    H = w[P + "decoder.rnn.weight_hh"].shape[1]
    ids = []
    for part in ("W", "R", "B"):
        counter[0] += 1
        ids.append(f"onnx::LSTM_{counter[0]}")
    Wt = onnx_gates(w[P + "decoder.rnn.weight_ih"], H)[None]
    Rt = onnx_gates(w[P + "decoder.rnn.weight_hh"], H)[None]
    Bt = np.concatenate([onnx_gates(w[P + "decoder.rnn.bias_ih"], H),
                         onnx_gates(w[P + "decoder.rnn.bias_hh"], H)])[None]
    inits += [tensor_proto(ids[0], Wt, FLOAT), tensor_proto(ids[1], Rt, FLOAT), tensor_proto(ids[2], Bt, FLOAT)]
    nodes.append(node("LSTM", [cur, ids[0], ids[1], ids[2], "", "h0", "c0"], [f"{tag}y", f"{tag}h", f"{tag}c"],
                      f"/{tag}decoder/rnn/LSTM", [attr_int("hidden_size", H)]))
    nodes.append(node("Relu", [f"{tag}h"], [f"{tag}hr"], f"/{tag}decoder/decoder/1/Relu"))
    dw, db = P + "decoder.decoder.2.weight", P + "decoder.decoder.2.bias"
    dwn, dbn = (tag + dw, tag + db) if tag else (dw, db)
    inits += [tensor_proto(dwn, w[dw], FLOAT), tensor_proto(dbn, w[db], FLOAT)]
    nodes.append(node("Conv", [f"{tag}hr", dwn, dbn], [f"{tag}o"], f"/{tag}decoder/decoder/2/Conv",
                      [attr_ints("kernel_shape", [1])]))
    nodes.append(node("Sigmoid", [f"{tag}o"], ["output" if not tag else f"{tag}out"], f"/{tag}decoder/decoder/3/Sigmoid"))
    return nodes, inits


def silero_8k_weights(seed: int) -> Dict[str, np.ndarray]:
    """The 8 kHz branch's parameters (basis [130][1][128], 65 bins) -- decoys the reader must
    pass over."""
    rng = np.random.default_rng(seed)
    P = "_model."
    w = {P + "stft.forward_basis_buffer": rng.normal(size=(130, 1, 128)).astype(np.float32)}
    cin = 65
    for i, co in enumerate((128, 64, 64, 128)):
        w[P + f"encoder.{i}.reparam_conv.weight"] = rng.normal(size=(co, cin, 3)).astype(np.float32)
        w[P + f"encoder.{i}.reparam_conv.bias"] = rng.normal(size=(co,)).astype(np.float32)
        cin = co
    for n, s in (("weight_ih", (512, 128)), ("weight_hh", (512, 128)), ("bias_ih", (512,)), ("bias_hh", (512,))):
        w[P + "decoder.rnn." + n] = rng.normal(size=s).astype(np.float32)
    w[P + "decoder.decoder.2.weight"] = rng.normal(size=(1, 128, 1)).astype(np.float32)
    w[P + "decoder.decoder.2.bias"] = rng.normal(size=(1,)).astype(np.float32)
    return w


def write_silero(dirpath: str, w: Dict[str, np.ndarray], variant: str = "flat",
                 name: str = "silero_vad_16k_op15.onnx") -> str:
    os.makedirs(dirpath, exist_ok=True)
    counter = [200]
    if variant == "flat":
        nodes, inits = silero_graph(w, "", False, counter)
        return write_model(os.path.join(dirpath, name), nodes, inits)
    n8, i8 = silero_graph(silero_8k_weights(5), "m8k/", False, counter)
    n16, i16 = silero_graph(w, "", True, counter)
    top = [node("Equal", ["sr", "c8000"], ["is8k"], "/Equal"),
           node("If", ["is8k"], ["output"], "/If",
                [attr_graph("then_branch", graph_proto(n8, i8, "then")),
                 attr_graph("else_branch", graph_proto(n16, i16, "else"))])]
    return write_model(os.path.join(dirpath, name), top, [])


# ------------------------------------------------------------------------------ CAM++
CONV_BN = [("head.conv1", "head.bn1"), ("head.conv2", "head.bn2"),
           ("xvector.tdnn.linear", "xvector.tdnn.nonlinear.batchnorm")]


def campp_conv_bn_pairs(w: Dict[str, np.ndarray]):
    pairs = list(CONV_BN)
    for n in w:
        if n.startswith("head.layer") and n.endswith((".conv1.weight", ".conv2.weight")):
            m = n[:-len(".weight")]
            pairs.append((m, m[:-5] + ("bn1" if m.endswith("conv1") else "bn2")))
        elif n.startswith("head.layer") and n.endswith(".shortcut.0.weight"):
            m = n[:-len(".weight")]
            pairs.append((m, m[:-1] + "1"))
        elif ".tdnnd" in n and n.endswith(".linear1.weight") and "cam_layer" not in n:
            m = n[:-len(".weight")]
            pairs.append((m, m[:-len("linear1")] + "nonlinear2.batchnorm"))
    return pairs


def fold(w: Dict[str, np.ndarray], conv: str, bn: str):
    """eval Conv + BN -> (W', b') in float32, as the exporter folds them."""
    W = w[conv + ".weight"]
    s = (w[bn + ".weight"] / np.sqrt(w[bn + ".running_var"] + np.float32(BN_EPS))).astype(np.float32)
    Wf = (W * s.reshape((-1,) + (1,) * (W.ndim - 1))).astype(np.float32)
    bf = (w[bn + ".bias"] - w[bn + ".running_mean"] * s).astype(np.float32)
    return Wf, bf


def write_campp(dirpath: str, w: Dict[str, np.ndarray], fused: bool = True,
                name: str = "campplus_cn_en_common_200k.onnx"):
    """Returns (path, expected tensors the reader must produce)."""
    os.makedirs(dirpath, exist_ok=True)
    pairs = dict(campp_conv_bn_pairs(w)) if fused else {}
    expect = dict(w)
    nodes, inits, done = [], [], set()
    counter = [500]
    dil = {}
    for n in w:
        if "cam_layer.linear_local.weight" in n:
            bi = int(n.split(".block")[1].split(".")[0])
            dil[n[:-len(".weight")]] = (1, 2, 2)[bi - 1]
    for n, a in w.items():
        if not n.endswith(".weight") or a.ndim < 3:
            continue
        m = n[:-len(".weight")]
        scope = "/" + m.replace(".", "/") + "/Conv"
        attrs = [attr_ints("dilations", [dil.get(m, 1)] * (a.ndim - 2))]
        if m in pairs:
            bn = pairs[m]
            Wf, bf = fold(w, m, bn)
            counter[0] += 2
            wn, bn_name = f"onnx::Conv_{counter[0] - 1}", f"onnx::Conv_{counter[0]}"
            inits += [tensor_proto(wn, Wf, FLOAT), tensor_proto(bn_name, bf, FLOAT)]
            nodes.append(node("Conv", ["x", wn, bn_name], [m + "_y"], scope, attrs))
            for k in ("weight", "bias", "running_mean", "running_var"):
                expect.pop(bn + "." + k, None)
                done.add(bn + "." + k)
            expect[n] = Wf
            expect[bn + ".fused_shift"] = bf
            done.add(n)
        else:
            ins = ["x", n] + ([m + ".bias"] if m + ".bias" in w else [])
            nodes.append(node("Conv", ins, [m + "_y"], scope, attrs))
    for n, a in w.items():
        if n in done:
            continue
        inits.append(tensor_proto(n, a, FLOAT))
    # BatchNormalization nodes of the BNs left in the graph (named parameters)
    for n in w:
        if n.endswith(".running_mean") and n not in done:
            m = n[:-len(".running_mean")]
            sc = m + ".weight" if m + ".weight" in w else "ones"
            bb = m + ".bias" if m + ".bias" in w else "zeros"
            nodes.append(node("BatchNormalization", ["x", sc, bb, n, m + ".running_var"], [m + "_y"],
                              "/" + m.replace(".", "/") + "/BatchNormalization"))
    return write_model(os.path.join(dirpath, name), nodes, inits), expect


# ------------------------------------------------------------------------------ ViBERT
def write_vibert(dirpath: str, w: Dict[str, np.ndarray], int8: bool = False,
                 name: str = None):
    """Returns (path, expected tensors)."""
    os.makedirs(dirpath, exist_ok=True)
    name = name or ("vibert-capu.int8.onnx" if int8 else "vibert-capu.onnx")
    nodes, inits = [], []
    expect = {}
    counter = [1000]
    for n, a in w.items():
        if n.endswith(".weight") and a.ndim == 2 and "embeddings" not in n:
            counter[0] += 1
            gen = f"onnx::MatMul_{counter[0]}"
            m = "model." + n[:-len(".weight")]
            scope = "/" + m.replace(".", "/") + "/MatMul"
            wt = np.ascontiguousarray(a.T)
            if int8:
                q, sc, zp = quantize(wt)
                inits += [tensor_proto(gen + "_quantized", q, INT8),
                          tensor_proto(gen + "_scale", np.array(sc, np.float32), FLOAT),
                          tensor_proto(gen + "_zero_point", np.array(zp, np.int8), INT8)]
                nodes.append(node("MatMulInteger", ["x_q", gen + "_quantized", "x_zp", gen + "_zero_point"],
                                  [gen + "_o"], scope + "_quant"))
                expect[n] = np.ascontiguousarray(((q.astype(np.float32) - np.float32(zp)) * sc).T)
            else:
                inits.append(tensor_proto(gen, wt, FLOAT))
                nodes.append(node("MatMul", ["x", gen], [gen + "_o"], scope))
                expect[n] = a
            nodes.append(node("Add", [gen + "_o", m + ".bias"], [gen + "_b"], scope[:-6] + "Add"))
        else:
            inits.append(tensor_proto("model." + n, a, FLOAT))
            expect[n] = a
    # buffers the export keeps (int64 position ids) are ignored by the reader
    inits.append(tensor_proto("model.bert.embeddings.position_ids",
                              np.arange(8, dtype=np.float32)[None], FLOAT))
    return write_model(os.path.join(dirpath, name), nodes, inits), expect
