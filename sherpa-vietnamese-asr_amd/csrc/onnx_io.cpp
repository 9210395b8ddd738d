// ONNX initializer reader (protobuf wire format, onnx.proto field numbers) and the mapping of
// a reference model directory onto the engine's weight names.  See onnx_io.h.
#include "onnx_io.h"

#include <dirent.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <stdexcept>

namespace zasr {

namespace {

// ---------------------------------------------------------------- protobuf wire format
struct Span {
  const uint8_t* p = nullptr;
  size_t n = 0;
  std::string str() const { return std::string(reinterpret_cast<const char*>(p), n); }
};

struct Pb {
  const uint8_t* p;
  const uint8_t* end;
  explicit Pb(Span s) : p(s.p), end(s.p + s.n) {}
  bool more() const { return p < end; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
      if (p >= end) throw std::runtime_error("onnx: truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
    throw std::runtime_error("onnx: bad varint");
  }
  void key(uint32_t& field, uint32_t& wire) {
    const uint64_t k = varint();
    field = (uint32_t)(k >> 3);
    wire = (uint32_t)(k & 7);
  }
  Span bytes() {
    const uint64_t n = varint();
    if (n > (uint64_t)(end - p)) throw std::runtime_error("onnx: truncated field");
    Span s{p, (size_t)n};
    p += n;
    return s;
  }
  // fixed-width field (wire types 1 and 5): checked before the pointer moves
  const uint8_t* fixed(size_t n) {
    if ((size_t)(end - p) < n) throw std::runtime_error("onnx: truncated field");
    const uint8_t* q = p;
    p += n;
    return q;
  }
  void skip(uint32_t wire) {
    switch (wire) {
      case 0: varint(); break;
      case 1: fixed(8); break;
      case 2: bytes(); break;
      case 5: fixed(4); break;
      default: throw std::runtime_error("onnx: unsupported wire type");
    }
  }
};

// onnx.proto TensorProto.DataType
enum { T_FLOAT = 1, T_UINT8 = 2, T_INT8 = 3, T_INT32 = 6, T_INT64 = 7, T_FLOAT16 = 10,
       T_DOUBLE = 11, T_BFLOAT16 = 16 };

struct RawTensor {
  std::string name;
  std::vector<int64_t> dims;
  int dtype = 0;
  Span raw;                  // raw_data (field 9)
  std::vector<float> f32;    // float_data (field 4)
  std::vector<int64_t> ints; // int32_data (5) / int64_data (7)
  std::string ext_location;  // external data (fields 13 / 14)
  long ext_offset = 0, ext_length = -1;
};

struct Node {
  std::string name, op;
  std::vector<std::string> in, out;
  std::map<std::string, std::vector<int64_t>> ints;  // int / ints attributes (strides, ...)
};

struct OnnxFile {
  std::string bytes;  // the whole file
  std::vector<RawTensor> inits;
  std::vector<Node> nodes;  // the main graph's, then each subgraph's (If branches) after its node
};

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  uint32_t bits;
  if (e == 0) {
    if (m == 0) {
      bits = s;
    } else {  // subnormal
      int ee = -1;
      uint32_t mm = m;
      do {
        ++ee;
        mm <<= 1;
      } while (!(mm & 0x400));
      bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3ff) << 13);
    }
  } else if (e == 31) {
    bits = s | 0x7f800000u | (m << 13);
  } else {
    bits = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  std::memcpy(&f, &bits, 4);
  return f;
}

RawTensor parse_tensor(Span s) {
  RawTensor t;
  Pb pb(s);
  while (pb.more()) {
    uint32_t f, w;
    pb.key(f, w);
    if (f == 1) {  // dims (packed or not)
      if (w == 2) {
        Pb q(pb.bytes());
        while (q.more()) t.dims.push_back((int64_t)q.varint());
      } else {
        t.dims.push_back((int64_t)pb.varint());
      }
    } else if (f == 2 && w == 0) {
      t.dtype = (int)pb.varint();
    } else if (f == 4) {  // float_data
      if (w == 2) {
        Span b = pb.bytes();
        const size_t k = b.n / 4;
        t.f32.resize(k);
        std::memcpy(t.f32.data(), b.p, k * 4);
      } else if (w == 5) {
        float v;
        std::memcpy(&v, pb.fixed(4), 4);
        t.f32.push_back(v);
      } else {
        pb.skip(w);
      }
    } else if ((f == 5 || f == 7) && (w == 2 || w == 0)) {  // int32_data / int64_data
      if (w == 2) {
        Pb q(pb.bytes());
        while (q.more()) t.ints.push_back((int64_t)q.varint());
      } else {
        t.ints.push_back((int64_t)pb.varint());
      }
    } else if (f == 8 && w == 2) {
      t.name = pb.bytes().str();
    } else if (f == 9 && w == 2) {
      t.raw = pb.bytes();
    } else if (f == 13 && w == 2) {  // external_data: StringStringEntryProto {1 key, 2 value}
      Pb q(pb.bytes());
      std::string k, v;
      while (q.more()) {
        uint32_t f2, w2;
        q.key(f2, w2);
        if (f2 == 1 && w2 == 2) k = q.bytes().str();
        else if (f2 == 2 && w2 == 2) v = q.bytes().str();
        else q.skip(w2);
      }
      try {
        if (k == "location") t.ext_location = v;
        else if (k == "offset") t.ext_offset = std::stol(v);
        else if (k == "length") t.ext_length = std::stol(v);
      } catch (const std::logic_error&) {
        throw std::runtime_error("onnx: bad external_data " + k + " '" + v + "'");
      }
    } else {
      pb.skip(w);
    }
  }
  return t;
}

// GraphProto: nodes (1) and initializers (5); subgraphs of node attributes (If / Loop
// branches: AttributeProto.g 6, .graphs 11) are flattened after their node, and Constant nodes'
// tensors (AttributeProto.t 5 of "value") count as initializers named by the node's output
void parse_graph(Span s, OnnxFile& of, int depth);

void parse_node(Span s, OnnxFile& of, int depth) {
  Node n;
  std::vector<Span> subgraphs;
  std::vector<RawTensor> consts;
  Pb pb(s);
  while (pb.more()) {
    uint32_t f, w;
    pb.key(f, w);
    if (w == 2 && f == 1) {
      n.in.push_back(pb.bytes().str());
    } else if (w == 2 && f == 2) {
      n.out.push_back(pb.bytes().str());
    } else if (w == 2 && f == 3) {
      n.name = pb.bytes().str();
    } else if (w == 2 && f == 4) {
      n.op = pb.bytes().str();
    } else if (w == 2 && f == 5) {  // AttributeProto
      Pb a(pb.bytes());
      std::string an;
      std::vector<int64_t> iv;
      bool has_int = false;
      while (a.more()) {
        uint32_t af, aw;
        a.key(af, aw);
        if (af == 1 && aw == 2) {
          an = a.bytes().str();
        } else if (af == 3 && aw == 0) {
          iv.push_back((int64_t)a.varint());
          has_int = true;
        } else if (af == 8) {
          has_int = true;
          if (aw == 2) {
            Pb q(a.bytes());
            while (q.more()) iv.push_back((int64_t)q.varint());
          } else {
            iv.push_back((int64_t)a.varint());
          }
        } else if (af == 5 && aw == 2) {
          consts.push_back(parse_tensor(a.bytes()));
        } else if ((af == 6 || af == 11) && aw == 2) {
          subgraphs.push_back(a.bytes());
        } else {
          a.skip(aw);
        }
      }
      if (has_int && !an.empty()) n.ints[an] = iv;
    } else {
      pb.skip(w);
    }
  }
  if (n.op == "Constant" && !n.out.empty())
    for (auto& t : consts) {
      t.name = n.out[0];
      of.inits.push_back(std::move(t));
    }
  of.nodes.push_back(std::move(n));
  for (const Span& g : subgraphs) parse_graph(g, of, depth + 1);
}

void parse_graph(Span s, OnnxFile& of, int depth) {
  if (depth > 8) throw std::runtime_error("onnx: subgraphs nested too deeply");
  Pb g(s);
  while (g.more()) {
    uint32_t gf, gw;
    g.key(gf, gw);
    if (gf == 1 && gw == 2) parse_node(g.bytes(), of, depth);
    else if (gf == 5 && gw == 2) of.inits.push_back(parse_tensor(g.bytes()));
    else g.skip(gw);
  }
}

void parse_file(const std::string& path, OnnxFile& of) {
  of.bytes = read_file(path);
  Span all{reinterpret_cast<const uint8_t*>(of.bytes.data()), of.bytes.size()};
  Pb model(all);
  bool have_graph = false;
  while (model.more()) {
    uint32_t f, w;
    model.key(f, w);
    if (f == 7 && w == 2) {  // ModelProto.graph
      have_graph = true;
      parse_graph(model.bytes(), of, 0);
    } else {
      model.skip(w);
    }
  }
  if (!have_graph) throw std::runtime_error("onnx: no graph in " + path);
}

// element count; negative dims or a count beyond 2^40 (a corrupt header) are errors, not a
// huge allocation
size_t numel_of(const std::vector<int64_t>& d) {
  size_t n = 1;
  for (int64_t x : d) {
    if (x < 0) throw std::runtime_error("onnx: negative tensor dimension");
    if (x != 0 && n > ((size_t)1 << 40) / (size_t)x)
      throw std::runtime_error("onnx: tensor too large");
    n *= (size_t)x;
  }
  return n;
}

// external data must stay inside the model directory: a relative path without '..'
void check_ext_location(const std::string& loc) {
  if (loc.empty() || loc[0] == '/' || loc[0] == '\\')
    throw std::runtime_error("onnx: external data location must be relative: " + loc);
  size_t a = 0;
  while (a <= loc.size()) {
    size_t b = loc.find_first_of("/\\", a);
    if (b == std::string::npos) b = loc.size();
    if (loc.compare(a, b - a, "..") == 0 && b - a == 2)
      throw std::runtime_error("onnx: external data location leaves the model directory: " + loc);
    a = b + 1;
  }
}

// the tensor's values as f32 (float / double / half / bfloat16 / int8 / uint8 / int32 / int64)
std::vector<float> to_f32(const RawTensor& t, const std::string& dir) {
  const size_t n = numel_of(t.dims);
  std::vector<float> out(n);
  std::string ext;
  Span raw = t.raw;
  if (!t.ext_location.empty()) {
    check_ext_location(t.ext_location);
    ext = read_file(dir + "/" + t.ext_location);
    const long len = t.ext_length >= 0 ? t.ext_length : (long)ext.size() - t.ext_offset;
    if (t.ext_offset < 0 || t.ext_offset + len > (long)ext.size())
      throw std::runtime_error("onnx: external data out of range for " + t.name);
    raw = Span{reinterpret_cast<const uint8_t*>(ext.data()) + t.ext_offset, (size_t)len};
  }
  auto need = [&](size_t bytes) {
    if (raw.n != bytes)
      throw std::runtime_error("onnx: raw_data size mismatch for " + t.name);
  };
  if (raw.n > 0) {
    switch (t.dtype) {
      case T_FLOAT: need(n * 4); std::memcpy(out.data(), raw.p, n * 4); break;
      case T_DOUBLE:
        need(n * 8);
        for (size_t i = 0; i < n; ++i) {
          double v;
          std::memcpy(&v, raw.p + 8 * i, 8);
          out[i] = (float)v;
        }
        break;
      case T_FLOAT16:
        need(n * 2);
        for (size_t i = 0; i < n; ++i) {
          uint16_t h;
          std::memcpy(&h, raw.p + 2 * i, 2);
          out[i] = half_to_float(h);
        }
        break;
      case T_BFLOAT16:
        need(n * 2);
        for (size_t i = 0; i < n; ++i) {
          uint16_t h;
          std::memcpy(&h, raw.p + 2 * i, 2);
          const uint32_t bits = (uint32_t)h << 16;
          std::memcpy(&out[i], &bits, 4);
        }
        break;
      case T_INT8: need(n); for (size_t i = 0; i < n; ++i) out[i] = (float)(int8_t)raw.p[i]; break;
      case T_UINT8: need(n); for (size_t i = 0; i < n; ++i) out[i] = (float)raw.p[i]; break;
      case T_INT32:
        need(n * 4);
        for (size_t i = 0; i < n; ++i) {
          int32_t v;
          std::memcpy(&v, raw.p + 4 * i, 4);
          out[i] = (float)v;
        }
        break;
      case T_INT64:
        need(n * 8);
        for (size_t i = 0; i < n; ++i) {
          int64_t v;
          std::memcpy(&v, raw.p + 8 * i, 8);
          out[i] = (float)v;
        }
        break;
      default:
        throw std::runtime_error("onnx: unsupported data type " + std::to_string(t.dtype) + " for " + t.name);
    }
  } else if (!t.f32.empty()) {
    if (t.f32.size() != n) throw std::runtime_error("onnx: float_data size mismatch for " + t.name);
    out = t.f32;
  } else if (!t.ints.empty()) {
    if (t.ints.size() != n) throw std::runtime_error("onnx: int data size mismatch for " + t.name);
    for (size_t i = 0; i < n; ++i) out[i] = (float)t.ints[i];
  } else if (n != 0) {
    throw std::runtime_error("onnx: tensor without data: " + t.name);
  }
  return out;
}

bool ends_with(const std::string& s, const std::string& x) {
  return s.size() >= x.size() && s.compare(s.size() - x.size(), x.size(), x) == 0;
}

// torch.onnx scope path of a node ("/encoder/encoders.0/layers.1/feed_forward1/in_proj/MatMul")
// -> module path ("encoder.encoders.0.layers.1.feed_forward1.in_proj")
std::string scope_module(const std::string& node_name) {
  if (node_name.empty() || node_name[0] != '/') return "";
  std::string s = node_name.substr(1);
  const size_t last = s.rfind('/');
  if (last == std::string::npos) return "";
  s = s.substr(0, last);
  std::replace(s.begin(), s.end(), '/', '.');
  return s;
}

struct Loaded {
  std::vector<int64_t> dims;
  std::vector<float> data;
};

// every initializer of a file as f32 under its own name, "<w>_quantized" int8 / uint8 tensors
// dequantized with "<w>_scale" and "<w>_zero_point" into "<w>" (onnxruntime quantize_dynamic:
// per-tensor scale; per-channel along the last axis)
std::map<std::string, Loaded> all_values(const OnnxFile& of, const std::string& dir) {
  std::map<std::string, const RawTensor*> byname;
  for (const auto& t : of.inits) byname[t.name] = &t;
  std::map<std::string, Loaded> vals;
  std::set<std::string> consumed;
  for (const auto& t : of.inits) {
    if (!ends_with(t.name, "_quantized")) continue;
    const std::string b = t.name.substr(0, t.name.size() - 10);
    auto sc = byname.find(b + "_scale"), zp = byname.find(b + "_zero_point");
    if (sc == byname.end()) continue;
    std::vector<float> q = to_f32(t, dir), s = to_f32(*sc->second, dir);
    std::vector<float> z = zp != byname.end() ? to_f32(*zp->second, dir) : std::vector<float>(s.size(), 0.f);
    if (s.empty() || z.size() != s.size()) throw std::runtime_error("onnx: bad quantization parameters for " + b);
    const size_t last = t.dims.empty() ? 1 : (size_t)t.dims.back();
    if (s.size() != 1 && s.size() != last)
      throw std::runtime_error("onnx: unsupported quantization axis for " + b);
    for (size_t i = 0; i < q.size(); ++i) {
      const size_t c = s.size() == 1 ? 0 : i % last;
      q[i] = (q[i] - z[c]) * s[c];
    }
    vals[b] = Loaded{t.dims, std::move(q)};
    consumed.insert(t.name);
    consumed.insert(b + "_scale");
    if (zp != byname.end()) consumed.insert(b + "_zero_point");
  }
  for (const auto& t : of.inits)
    if (!consumed.count(t.name) && !vals.count(t.name)) vals[t.name] = Loaded{t.dims, to_f32(t, dir)};
  return vals;
}

// one file's initializers under the names the engine uses; MatMul weights that neither a scope
// name nor a following bias names are appended to `unnamed` in graph (execution) order
void map_file(const OnnxFile& of, const std::string& dir, const std::string& prefix,
              std::map<std::string, Loaded>& out, std::vector<Loaded>* unnamed) {
  // 1. every initializer, int8 weights dequantized
  std::map<std::string, Loaded> vals = all_values(of, dir);
  // 2. MatMul / MatMulInteger weight operands: the exporter stores nn.Linear weights
  //    transposed ([in][out]) under generated names; name them from the node's scope path, or
  //    from the bias of the Add that follows (through Cast / Mul for MatMulInteger)
  std::map<std::string, std::vector<const Node*>> consumers;
  for (const auto& n : of.nodes)
    for (const auto& i : n.in) consumers[i].push_back(&n);
  auto base_of = [](const std::string& x) {
    return ends_with(x, "_quantized") ? x.substr(0, x.size() - 10) : x;
  };
  std::map<std::string, std::string> rename;  // generated name -> module weight name
  for (const auto& n : of.nodes) {
    if ((n.op != "MatMul" && n.op != "MatMulInteger") || n.in.size() < 2) continue;
    const std::string w = base_of(n.in[1]);
    if (!vals.count(w) || vals[w].dims.size() != 2 || ends_with(w, ".weight")) continue;
    std::string mod = scope_module(n.name);
    if (mod.empty() && !n.out.empty()) {  // follow the output to an Add with a named bias
      std::string cur = n.out[0];
      for (int hop = 0; hop < 4 && mod.empty(); ++hop) {
        const Node* nxt = nullptr;
        for (const Node* c : consumers[cur]) {
          if (c->op == "Add") {
            for (const auto& i : c->in)
              if (ends_with(i, ".bias") && vals.count(i)) mod = i.substr(0, i.size() - 5);
          }
          if (c->op == "Cast" || c->op == "Mul") nxt = c;
        }
        if (!nxt || nxt->out.empty()) break;
        cur = nxt->out[0];
      }
    }
    if (!mod.empty()) {
      rename[w] = mod + ".weight";
    } else if (unnamed) {
      unnamed->push_back(vals[w]);
      vals.erase(w);
    }
  }
  for (const auto& kv : rename) {
    Loaded& l = vals[kv.first];
    const int64_t K = l.dims[0], N = l.dims[1];
    Loaded t{{N, K}, std::vector<float>(l.data.size())};
    for (int64_t k = 0; k < K; ++k)
      for (int64_t c = 0; c < N; ++c) t.data[(size_t)c * K + k] = l.data[(size_t)k * N + c];
    out[prefix + kv.second] = std::move(t);
  }
  for (auto& kv : vals) {
    if (rename.count(kv.first)) continue;
    if (kv.first.rfind("onnx::", 0) == 0 || kv.first.empty()) continue;  // graph constants
    std::string name = kv.first;
    if (name.rfind(prefix, 0) != 0) name = prefix + name;
    if (!out.count(name)) out[name] = std::move(kv.second);
  }
}

int dim(const std::map<std::string, Loaded>& w, const std::string& name, size_t axis) {
  auto it = w.find(name);
  if (it == w.end()) throw std::runtime_error("onnx model: missing tensor " + name);
  if (axis >= it->second.dims.size()) throw std::runtime_error("onnx model: bad rank for " + name);
  return (int)it->second.dims[axis];
}

std::string ivec(const std::vector<int>& v) {
  std::ostringstream os;
  os << "[";
  for (size_t i = 0; i < v.size(); ++i) os << (i ? ", " : "") << v[i];
  os << "]";
  return os.str();
}

// ZipformerConfig (zasr/model.py) from the tensor shapes; query / positional head dims are the
// kernels' 32 / 4
std::string infer_config(const std::map<std::string, Loaded>& w) {
  std::vector<int> dims, layers, ff, heads, ds, kernels;
  int vd = 0, pos_dim = 0;
  for (int i = 0;; ++i) {
    const std::string s = "encoder.encoders." + std::to_string(i) + ".";
    const bool down = w.count(s + "downsample.bias") != 0;
    const std::string pre = s + (down ? "encoder." : "");
    if (!w.count(pre + "layers.0.norm.bias")) break;
    int nl = 0;
    while (w.count(pre + "layers." + std::to_string(nl) + ".norm.bias")) ++nl;
    const std::string L = pre + "layers.0.";
    const int d = dim(w, L + "norm.bias", 0);
    const int h = dim(w, L + "self_attn_weights.in_proj.weight", 0) / (2 * 32 + 4);
    dims.push_back(d);
    layers.push_back(nl);
    ff.push_back(dim(w, L + "feed_forward2.in_proj.weight", 0));
    heads.push_back(h);
    ds.push_back(down ? dim(w, s + "downsample.bias", 0) : 1);
    kernels.push_back(dim(w, L + "conv_module1.depthwise_conv.weight", 2));
    vd = dim(w, L + "self_attn1.in_proj.weight", 0) / h;
    pos_dim = dim(w, L + "self_attn_weights.linear_pos.weight", 1);
  }
  if (dims.empty()) throw std::runtime_error("onnx model: no Zipformer2 encoder stacks found");
  std::ostringstream os;
  os << "{\"name\": \"zipformer-onnx\", \"encoder_dims\": " << ivec(dims)
     << ", \"num_layers\": " << ivec(layers) << ", \"ff_dims\": " << ivec(ff)
     << ", \"num_heads\": " << ivec(heads) << ", \"downsampling\": " << ivec(ds)
     << ", \"cnn_kernels\": " << ivec(kernels) << ", \"query_head_dim\": 32"
     << ", \"value_head_dim\": " << vd << ", \"pos_head_dim\": 4, \"pos_dim\": " << pos_dim
     << ", \"vocab_size\": " << dim(w, "joiner.output_linear.weight", 0)
     << ", \"decoder_dim\": " << dim(w, "decoder.embedding.weight", 1)
     << ", \"joiner_dim\": " << dim(w, "joiner.output_linear.weight", 1)
     << ", \"context_size\": " << dim(w, "decoder.conv.weight", 2)
     << ", \"layer1_channels\": " << dim(w, "encoder_embed.conv.0.weight", 0)
     << ", \"layer2_channels\": " << dim(w, "encoder_embed.conv.4.weight", 0)
     << ", \"layer3_channels\": " << dim(w, "encoder_embed.conv.7.weight", 0) << "}";
  return os.str();
}


// ------------------------------------------------------------ single-graph stage models
const Loaded* input_value(const std::map<std::string, Loaded>& v, const Node& n, size_t i) {
  if (i >= n.in.size()) return nullptr;
  auto it = v.find(n.in[i]);
  return it == v.end() ? nullptr : &it->second;
}

int64_t attr0(const Node& n, const std::string& k, int64_t dflt) {
  auto it = n.ints.find(k);
  return it == n.ints.end() || it->second.empty() ? dflt : it->second[0];
}

// ONNX LSTM gate blocks (i, o, f, c) -> torch LSTMCell (i, f, g, o) rows of [4H][K]
std::vector<float> lstm_gates_to_torch(const float* src, int64_t H, int64_t K) {
  static const int from[4] = {0, 2, 3, 1};
  std::vector<float> out((size_t)(4 * H * K));
  for (int g = 0; g < 4; ++g)
    std::memcpy(out.data() + (size_t)g * H * K, src + (size_t)from[g] * H * K, (size_t)(H * K) * 4);
  return out;
}

// Silero VAD v5, 16 kHz branch (silero_vad_16k_op15.onnx / silero_vad.onnx, core/vad_utils.py:
// 22-24).  The graph is walked, not its names: the STFT Conv (basis [258][1][256]; an 8 kHz
// branch's [130][1][128] is passed over), the kernel-3 Convs chained from 129 channels up to
// the LSTM (strides from their attributes), the LSTM node (W / R / B, ONNX gate order iofc,
// reordered to torch's ifgo) or named decoder.rnn.* tensors, then the [1][H][1] output Conv.
// Every subgraph is flattened (an If on the sample rate keeps its branches there).
std::string load_silero_graph(const OnnxFile& of, const std::string& dir, SafeTensors& out) {
  const auto v = all_values(of, dir);
  const size_t N = of.nodes.size();
  size_t at = N;
  for (size_t k = 0; k < N && at == N; ++k) {
    const Node& n = of.nodes[k];
    const Loaded* w = n.op == "Conv" ? input_value(v, n, 1) : nullptr;
    if (w && w->dims.size() == 3 && w->dims[0] == 258 && w->dims[1] == 1 && w->dims[2] == 256) at = k;
  }
  if (at == N) throw std::runtime_error("silero onnx: no 16 kHz STFT Conv (basis [258][1][256])");
  const std::string P = "_model.";
  out.put(P + "stft.forward_basis_buffer", {258, 1, 256}, std::vector<float>(input_value(v, of.nodes[at], 1)->data));
  std::vector<int> ch, sd;
  int64_t cin = 129;
  size_t k = at + 1;
  for (; k < N && of.nodes[k].op != "LSTM"; ++k) {
    const Node& n = of.nodes[k];
    const Loaded* w = n.op == "Conv" ? input_value(v, n, 1) : nullptr;
    if (!w || w->dims.size() != 3 || w->dims[2] != 3 || w->dims[1] != cin) continue;
    const int64_t co = w->dims[0];
    const std::string L = P + "encoder." + std::to_string(ch.size()) + ".reparam_conv.";
    out.put(L + "weight", w->dims, std::vector<float>(w->data));
    const Loaded* b = input_value(v, n, 2);
    if (b && (int64_t)b->data.size() != co) throw std::runtime_error("silero onnx: bad encoder bias");
    out.put(L + "bias", {co}, b ? std::vector<float>(b->data) : std::vector<float>((size_t)co, 0.f));
    ch.push_back((int)co);
    sd.push_back((int)attr0(n, "strides", 1));
    cin = co;
  }
  if (ch.empty()) throw std::runtime_error("silero onnx: no encoder Convs after the STFT");
  int64_t H = 0;
  if (k < N) {  // the LSTM node: X, W [1][4H][in], R [1][4H][H], B [1][8H]
    const Node& n = of.nodes[k];
    const Loaded *W = input_value(v, n, 1), *R = input_value(v, n, 2), *B = input_value(v, n, 3);
    if (!W || !R || W->dims.size() != 3 || R->dims.size() != 3 || W->dims[0] != 1 || W->dims[2] != cin)
      throw std::runtime_error("silero onnx: unsupported LSTM weights");
    H = R->dims[2];
    if (W->dims[1] != 4 * H || R->dims[1] != 4 * H) throw std::runtime_error("silero onnx: bad LSTM shapes");
    out.put(P + "decoder.rnn.weight_ih", {4 * H, cin}, lstm_gates_to_torch(W->data.data(), H, cin));
    out.put(P + "decoder.rnn.weight_hh", {4 * H, H}, lstm_gates_to_torch(R->data.data(), H, H));
    std::vector<float> bi((size_t)(4 * H), 0.f), bh((size_t)(4 * H), 0.f);
    if (B) {
      if ((int64_t)B->data.size() != 8 * H) throw std::runtime_error("silero onnx: bad LSTM bias");
      bi = lstm_gates_to_torch(B->data.data(), H, 1);
      bh = lstm_gates_to_torch(B->data.data() + 4 * H, H, 1);
    }
    out.put(P + "decoder.rnn.bias_ih", {4 * H}, std::move(bi));
    out.put(P + "decoder.rnn.bias_hh", {4 * H}, std::move(bh));
  } else {  // an export that keeps the LSTMCell parameters by name
    for (const char* nm : {"weight_ih", "weight_hh", "bias_ih", "bias_hh"}) {
      const Loaded* f = nullptr;
      for (const auto& kv : v)
        if (ends_with(kv.first, std::string("decoder.rnn.") + nm) && kv.first.find("8k") == std::string::npos) f = &kv.second;
      if (!f) throw std::runtime_error(std::string("silero onnx: no LSTM node and no decoder.rnn.") + nm);
      if (H == 0) H = f->dims[0] / 4;
      out.put(P + "decoder.rnn." + nm, f->dims, std::vector<float>(f->data));
    }
    k = at;
  }
  bool dec = false;
  for (size_t q = k + 1; q < N && !dec; ++q) {
    const Node& n = of.nodes[q];
    const Loaded* w = n.op == "Conv" ? input_value(v, n, 1) : nullptr;
    if (!w || w->dims.size() != 3 || w->dims[0] != 1 || w->dims[1] != H || w->dims[2] != 1) continue;
    const Loaded* b = input_value(v, n, 2);
    out.put(P + "decoder.decoder.2.weight", {1, H, 1}, std::vector<float>(w->data));
    out.put(P + "decoder.decoder.2.bias", {1}, b ? std::vector<float>(b->data) : std::vector<float>(1, 0.f));
    dec = true;
  }
  if (!dec) throw std::runtime_error("silero onnx: no output Conv [1][H][1] after the LSTM");
  std::ostringstream os;
  os << "{\"sample_rate\": 16000, \"window\": 512, \"context\": 64, \"filter_length\": 256, "
     << "\"hop\": " << attr0(of.nodes[at], "strides", 128) << ", \"enc_channels\": " << ivec(ch)
     << ", \"enc_strides\": " << ivec(sd) << ", \"hidden\": " << H << "}";
  return os.str();
}

// CAM++ (campplus_cn_en_common_200k.onnx, convert_onnx/export_campplus_onnx.py: torch.onnx,
// opset 17, constant folding, eval mode).  Tensors that keep their state-dict names are taken
// as they are; Conv and BatchNormalization nodes are named from their scope path
// ("/xvector/block1/tdnnd1/linear1/Conv").  A Conv that carries a bias where the state dict has
// a BatchNorm after it was fused by the exporter (W*s, beta - mean*s): its bias becomes
// "<bn>.fused_shift" and the engine applies the identity scale (campp.cpp bn_fold).
std::string bn_after_conv(const std::string& mod) {
  auto rep = [&](const std::string& a, const std::string& b) { return mod.substr(0, mod.size() - a.size()) + b; };
  if (mod.rfind("head.", 0) == 0) {
    if (ends_with(mod, "conv1")) return rep("conv1", "bn1");
    if (ends_with(mod, "conv2")) return rep("conv2", "bn2");
    if (ends_with(mod, "shortcut.0")) return rep("shortcut.0", "shortcut.1");
    return "";
  }
  if (mod == "xvector.tdnn.linear") return "xvector.tdnn.nonlinear.batchnorm";
  if (mod == "xvector.dense.linear") return "xvector.dense.nonlinear.batchnorm";
  if (mod.find(".tdnnd") != std::string::npos && mod.find("cam_layer") == std::string::npos &&
      ends_with(mod, ".linear1"))
    return rep("linear1", "nonlinear2.batchnorm");
  return "";
}

std::string load_campp_graph(const OnnxFile& of, const std::string& dir, SafeTensors& out) {
  const auto v = all_values(of, dir);
  std::map<std::string, Loaded> w;
  for (const auto& kv : v)
    if (kv.first.rfind("head.", 0) == 0 || kv.first.rfind("xvector.", 0) == 0) w[kv.first] = kv.second;
  std::set<std::string> bn_nodes;
  for (const Node& n : of.nodes) {
    const std::string mod = scope_module(n.name);
    if (n.op != "BatchNormalization" || mod.empty()) continue;
    bn_nodes.insert(mod);
    static const char* parts[] = {"weight", "bias", "running_mean", "running_var"};
    for (size_t i = 0; i < 4; ++i) {
      const Loaded* x = input_value(v, n, i + 1);
      if (x && !w.count(mod + "." + parts[i])) w[mod + "." + parts[i]] = *x;
    }
  }
  std::map<std::string, std::vector<int>> dil;  // Conv dilations by module (block kernels)
  for (const Node& n : of.nodes) {
    const std::string mod = scope_module(n.name);
    if (n.op != "Conv" || mod.empty()) continue;
    const Loaded* x = input_value(v, n, 1);
    if (x && !w.count(mod + ".weight")) w[mod + ".weight"] = *x;
    dil[mod] = {(int)attr0(n, "dilations", 1)};
    const Loaded* b = input_value(v, n, 2);
    if (!b) continue;
    const std::string bn = bn_after_conv(mod);
    if (!bn.empty() && !bn_nodes.count(bn) && !w.count(bn + ".running_mean")) {
      w[bn + ".fused_shift"] = *b;
    } else if (!w.count(mod + ".bias")) {
      w[mod + ".bias"] = *b;
    }
  }
  if (!w.count("xvector.tdnn.linear.weight") || !w.count("xvector.dense.linear.weight"))
    throw std::runtime_error("campp onnx: xvector.tdnn / xvector.dense Conv weights not found (scope names "
                             "or state-dict names needed)");
  std::vector<int> head, layers, kernels, dils;
  for (int l = 1; w.count("head.layer" + std::to_string(l) + ".0.conv1.weight"); ++l) {
    int nb = 0;
    while (w.count("head.layer" + std::to_string(l) + "." + std::to_string(nb) + ".conv1.weight")) ++nb;
    head.push_back(nb);
  }
  for (int b = 1; w.count("xvector.block" + std::to_string(b) + ".tdnnd1.linear1.weight"); ++b) {
    const std::string B = "xvector.block" + std::to_string(b) + ".tdnnd";
    int nl = 0;
    while (w.count(B + std::to_string(nl + 1) + ".linear1.weight")) ++nl;
    layers.push_back(nl);
    const std::string loc = B + "1.cam_layer.linear_local";
    kernels.push_back((int)w.at(loc + ".weight").dims.back());
    dils.push_back(dil.count(loc) ? dil[loc][0] : 1);
  }
  const Loaded& tdnn = w.at("xvector.tdnn.linear.weight");
  const Loaded& dense = w.at("xvector.dense.linear.weight");
  const Loaded& l1 = w.at("xvector.block1.tdnnd1.linear1.weight");
  const Loaded& loc1 = w.at("xvector.block1.tdnnd1.cam_layer.linear_local.weight");
  // the FCM head's output is m_channels x (feat_dim / 8) features (head.conv1's output
  // channels = m_channels): the TDNN input width divided by it, times 8
  const long m_channels = w.at("head.conv1.weight").dims[0];
  if (m_channels <= 0 || tdnn.dims[1] % m_channels != 0)
    throw std::runtime_error("CAM++ graph: TDNN input width " + std::to_string(tdnn.dims[1]) +
                             " is not a multiple of the head's m_channels " +
                             std::to_string(m_channels));
  std::ostringstream os;
  os << "{\"feat_dim\": " << tdnn.dims[1] / m_channels * 8 << ", \"embedding_size\": " << dense.dims[0]
     << ", \"growth_rate\": " << loc1.dims[0] << ", \"bn_size\": " << l1.dims[0] / loc1.dims[0]
     << ", \"init_channels\": " << tdnn.dims[0] << ", \"m_channels\": " << m_channels
     << ", \"head_blocks\": " << ivec(head) << ", \"block_layers\": " << ivec(layers)
     << ", \"block_kernels\": " << ivec(kernels) << ", \"block_dilations\": " << ivec(dils) << "}";
  for (auto& kv : w) out.put(kv.first, kv.second.dims, std::move(kv.second.data));
  return os.str();
}

// ViBERT-capu (vibert-capu.onnx / .int8.onnx, convert_onnx/export_vibert_onnx.py: the
// Seq2LabelsModel inside the _ViBERTForExport wrapper, so every name carries "model.").  Linear
// weights are named by map_file (scope path or bias Add) and transposed back; the head count
// and LayerNorm eps are not in the tensors: config.json's num_attention_heads /
// layer_norm_eps when the directory has them, else BERT's head dim 64 and 1e-12.
std::string load_vibert_graph(const OnnxFile& of, const std::string& dir, SafeTensors& out) {
  std::map<std::string, Loaded> m, w;
  map_file(of, dir, "", m, nullptr);
  for (auto& kv : m) {
    std::string n = kv.first;
    if (n.rfind("model.", 0) == 0) n = n.substr(6);
    const bool param = ends_with(n, ".weight") || ends_with(n, ".bias");  // not the id buffers
    if (param && (n.rfind("bert.", 0) == 0 || n.rfind("classifier.", 0) == 0 || n.rfind("detector.", 0) == 0))
      w[n] = std::move(kv.second);
  }
  const std::string E = "bert.embeddings.";
  const int H = dim(w, E + "word_embeddings.weight", 1);
  int layers = 0;
  while (w.count("bert.encoder.layer." + std::to_string(layers) + ".attention.self.query.weight")) ++layers;
  if (layers == 0) throw std::runtime_error("vibert onnx: no encoder layers found");
  int heads = H / 64;
  double eps = 1e-12;
  const std::string cj = dir + "/config.json";
  if (file_exists(cj)) {
    const Json j = Json::parse(read_file(cj));
    if (j.has("num_attention_heads")) heads = (int)j.at("num_attention_heads").num;
    if (j.has("layer_norm_eps")) eps = j.at("layer_norm_eps").num;
  }
  std::ostringstream os;
  os.precision(17);
  os << "{\"hidden_size\": " << H << ", \"num_hidden_layers\": " << layers
     << ", \"num_attention_heads\": " << heads
     << ", \"intermediate_size\": " << dim(w, "bert.encoder.layer.0.intermediate.dense.weight", 0)
     << ", \"max_position_embeddings\": " << dim(w, E + "position_embeddings.weight", 0)
     << ", \"type_vocab_size\": " << dim(w, E + "token_type_embeddings.weight", 0)
     << ", \"vocab_size\": " << dim(w, E + "word_embeddings.weight", 0)
     << ", \"num_labels\": " << dim(w, "classifier.weight", 0)
     << ", \"num_detect_classes\": " << dim(w, "detector.weight", 0) << ", \"layer_norm_eps\": " << eps << "}";
  for (auto& kv : w) out.put(kv.first, kv.second.dims, std::move(kv.second.data));
  return os.str();
}

}  // namespace

OnnxFiles find_onnx_files(const std::string& dir) {
  // core/asr_engine.py:913-928: the first directory entry starting with the pattern and ending
  // in .onnx whose name does not contain "int8"; else the first such file
  std::vector<std::string> names;
  if (DIR* d = opendir(dir.c_str())) {
    while (dirent* e = readdir(d)) names.push_back(e->d_name);
    closedir(d);
  }
  auto pick = [&](const std::string& pat) -> std::string {
    std::string any, flt;
    for (const auto& f : names) {
      if (f.rfind(pat, 0) != 0 || !ends_with(f, ".onnx")) continue;
      if (any.empty()) any = f;
      if (flt.empty() && f.find("int8") == std::string::npos) flt = f;
    }
    const std::string f = !flt.empty() ? flt : any;
    return f.empty() ? "" : dir + "/" + f;
  };
  return OnnxFiles{pick("encoder-"), pick("decoder-"), pick("joiner-")};
}

std::string load_onnx_model(const OnnxFiles& files, SafeTensors& out) {
  std::map<std::string, Loaded> w;
  std::vector<Loaded> unnamed;  // encoder MatMul weights without a scope name or bias
  const std::pair<const std::string*, const char*> parts[] = {
      {&files.encoder, ""}, {&files.decoder, ""}, {&files.joiner, "joiner."}};
  for (const auto& pr : parts) {
    OnnxFile of;
    parse_file(*pr.first, of);
    const std::string dir = pr.first->substr(0, pr.first->rfind('/'));
    std::map<std::string, Loaded> part;
    map_file(of, dir, pr.second, part, pr.first == &files.encoder ? &unnamed : nullptr);
    for (auto& kv : part) {
      // an exporter may keep encoder_proj / decoder_proj in the joiner graph
      std::string name = kv.first;
      if (name.rfind("joiner.encoder_proj.", 0) == 0 || name.rfind("joiner.decoder_proj.", 0) == 0)
        name = name.substr(7);
      if (!w.count(name)) w[name] = std::move(kv.second);
    }
  }
  // bias-free linears (self_attn_weights.linear_pos) of an export without scope names: in
  // execution order, layer by layer, each the next unnamed weight of shape [pos_dim][4 h]
  size_t next_unnamed = 0;
  for (int i = 0;; ++i) {
    const std::string s = "encoder.encoders." + std::to_string(i) + ".";
    const std::string pre = s + (w.count(s + "downsample.bias") ? "encoder." : "");
    if (!w.count(pre + "layers.0.norm.bias")) break;
    for (int j = 0; w.count(pre + "layers." + std::to_string(j) + ".norm.bias"); ++j) {
      const std::string L = pre + "layers." + std::to_string(j) + ".self_attn_weights.";
      if (w.count(L + "linear_pos.weight") || !w.count(L + "in_proj.weight")) continue;
      const int64_t n4 = 4 * (w[L + "in_proj.weight"].dims[0] / (2 * 32 + 4));
      while (next_unnamed < unnamed.size() && unnamed[next_unnamed].dims[1] != n4) ++next_unnamed;
      if (next_unnamed == unnamed.size()) break;
      const Loaded& u = unnamed[next_unnamed++];
      const int64_t K = u.dims[0], N = u.dims[1];
      Loaded t{{N, K}, std::vector<float>(u.data.size())};
      for (int64_t k = 0; k < K; ++k)
        for (int64_t c = 0; c < N; ++c) t.data[(size_t)c * K + k] = u.data[(size_t)k * N + c];
      w[L + "linear_pos.weight"] = std::move(t);
    }
  }
  const std::string cfg = infer_config(w);
  for (auto& kv : w) out.put(kv.first, kv.second.dims, std::move(kv.second.data));
  return cfg;
}

std::string load_model_dir(const std::string& dir, SafeTensors& out) {
  const std::string cfg_path = dir + "/config.json", st_path = dir + "/model.safetensors";
  if (file_exists(cfg_path) && file_exists(st_path)) {
    out.load(st_path);
    return read_file(cfg_path);
  }
  const OnnxFiles f = find_onnx_files(dir);
  if (f.complete()) {
    std::string cfg = load_onnx_model(f, out);
    if (file_exists(cfg_path)) cfg = read_file(cfg_path);  // an explicit config wins
    return cfg;
  }
  throw std::invalid_argument("missing model files in " + dir +
                              " (config.json + model.safetensors, or encoder-/decoder-/joiner-*.onnx)");
}

void write_safetensors(const std::string& path, const SafeTensors& t) {
  std::ostringstream hdr;
  hdr << "{";
  size_t off = 0;
  bool first = true;
  for (const auto& kv : t.all()) {
    hdr << (first ? "" : ",") << "\"" << kv.first << "\":{\"dtype\":\"F32\",\"shape\":[";
    for (size_t i = 0; i < kv.second.shape.size(); ++i) hdr << (i ? "," : "") << kv.second.shape[i];
    hdr << "],\"data_offsets\":[" << off << "," << off + kv.second.numel * 4 << "]}";
    off += kv.second.numel * 4;
    first = false;
  }
  hdr << "}";
  std::string h = hdr.str();
  while ((8 + h.size()) % 8) h += ' ';
  std::ofstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot write " + path);
  const uint64_t hl = h.size();
  f.write(reinterpret_cast<const char*>(&hl), 8);
  f.write(h.data(), (std::streamsize)h.size());
  for (const auto& kv : t.all())
    f.write(reinterpret_cast<const char*>(kv.second.data), (std::streamsize)(kv.second.numel * 4));
  if (!f) throw std::runtime_error("write failed: " + path);
}

std::string find_stage_onnx(const std::string& dir, const std::string& kind) {
  // the file names the reference opens (core/vad_utils.py:22-24, core/speaker_diarization_
  // senko_campp_optimized.py:324-325, core/gec_model.py:133-140: fp32 preferred)
  std::vector<std::string> cands;
  if (kind == "silero") cands = {"silero_vad_16k_op15.onnx", "silero_vad.onnx"};
  else if (kind == "campp") cands = {"campplus_cn_en_common_200k.onnx"};
  else if (kind == "vibert") cands = {"vibert-capu.onnx", "vibert-capu.int8.onnx"};
  else throw std::invalid_argument("unknown model kind " + kind);
  for (const auto& c : cands)
    if (file_exists(dir + "/" + c)) return dir + "/" + c;
  return "";
}

std::string load_stage_onnx(const std::string& path, const std::string& kind, SafeTensors& out) {
  OnnxFile of;
  parse_file(path, of);
  const std::string dir = path.substr(0, path.rfind('/') == std::string::npos ? 0 : path.rfind('/'));
  if (kind == "silero") return load_silero_graph(of, dir.empty() ? "." : dir, out);
  if (kind == "campp") return load_campp_graph(of, dir.empty() ? "." : dir, out);
  if (kind == "vibert") return load_vibert_graph(of, dir.empty() ? "." : dir, out);
  throw std::invalid_argument("unknown model kind " + kind);
}

std::string load_stage_dir(const std::string& dir, const std::string& kind, SafeTensors& out) {
  std::string cfg, st;
  if (kind == "silero") cfg = "silero_config.json", st = "silero_vad.safetensors";
  else if (kind == "campp") cfg = "campp_config.json", st = "campp.safetensors";
  else if (kind == "vibert") cfg = "vibert_config.json", st = "vibert.safetensors";
  else throw std::invalid_argument("unknown model kind " + kind);
  // the file itself, as the reference's create_ort_session callers name it
  // (core/speaker_diarization_senko_campp_optimized.py:322-325, core/gec_model.py:133-140)
  if (ends_with(dir, ".onnx") && file_exists(dir)) return load_stage_onnx(dir, kind, out);
  if (file_exists(dir + "/" + cfg) && file_exists(dir + "/" + st)) {
    out.load(dir + "/" + st);
    return read_file(dir + "/" + cfg);
  }
  const std::string f = find_stage_onnx(dir, kind);
  if (f.empty())
    throw std::invalid_argument("missing " + kind + " model files in " + dir + " (" + cfg + " + " + st +
                                ", or the reference's .onnx)");
  return load_stage_onnx(f, kind, out);
}

std::string stage_safetensors_name(const std::string& kind) {
  if (kind == "silero") return "silero_vad.safetensors";
  if (kind == "campp") return "campp.safetensors";
  if (kind == "vibert") return "vibert.safetensors";
  throw std::invalid_argument("unknown model kind " + kind);
}

}  // namespace zasr
