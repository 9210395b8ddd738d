// libzasr host runtime: model upload, fbank / encoder / search drivers.
//
// Reference mapping:
//   load + session setup    core/asr_engine.py:903-1020 (create_recognizer)
//   fbank                   core/asr_engine.py:698-721
//   encoder run             core/asr_engine.py:1045-1049 (Zipformer2 graph, icefall 3P)
//   search loop             core/asr_engine.py:1051-1153
#include "engine.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <deque>
#include <numeric>
#include <cstdlib>
#include <sstream>

#include "common.h"
#include "gemm.h"
#include "host_io.h"
#include "onnx_io.h"

namespace zasr {

// ------------------------------------------------------------------------------------
// hotwords: Aho-Corasick graph restated from core/hotword_context.py:46-184, flattened
// to a dense (state x trie-token) transition table of (next state, score delta)
// ------------------------------------------------------------------------------------
namespace {
struct HwNode {
  int tok = -1;
  double tok_score = 0, node_score = 0, out_score = 0;
  bool is_end = false;
  std::vector<std::pair<int, int>> kids;  // (token, node) in insertion order
  int fail = 0, out = -1;
  int child(int t) const {
    for (auto& k : kids)
      if (k.first == t) return k.second;
    return -1;
  }
};
}  // namespace

HotwordDFA build_hotword_dfa(const std::vector<std::vector<int>>& phrases,
                             const std::vector<float>& scores, int V) {
  HotwordDFA dfa;
  if (phrases.empty()) return dfa;
  std::vector<HwNode> nd(1);
  for (size_t p = 0; p < phrases.size(); ++p) {
    const auto& seq = phrases[p];
    if (seq.empty()) continue;
    double sc = (double)scores[p];
    int cur = 0;
    for (size_t j = 0; j < seq.size(); ++j) {
      int t = seq[j];
      ZASR_REQUIRE(t >= 0 && t < V, "hotword token id out of range");
      bool last = (j + 1 == seq.size());
      int c = nd[cur].child(t);
      if (c < 0) {
        HwNode n;
        n.tok = t;
        n.tok_score = sc;
        n.node_score = nd[cur].node_score + sc;
        n.out_score = last ? n.node_score : 0.0;
        n.is_end = last;
        nd.push_back(n);
        c = (int)nd.size() - 1;
        nd[cur].kids.push_back({t, c});
      } else {
        HwNode& e = nd[c];
        e.tok_score = std::max(sc, e.tok_score);
        e.node_score = nd[cur].node_score + e.tok_score;
        if (last) e.is_end = true;
        if (e.is_end) e.out_score = e.node_score;
      }
      cur = c;
    }
  }
  // BFS fail / output links
  std::deque<int> q;
  for (auto& k : nd[0].kids) {
    nd[k.second].fail = 0;
    q.push_back(k.second);
  }
  while (!q.empty()) {
    int cur = q.front();
    q.pop_front();
    for (auto& k : nd[cur].kids) {
      int t = k.first, kid = k.second;
      int f = nd[cur].fail;
      int c = nd[f].child(t);
      if (c >= 0) {
        f = c;
      } else {
        f = nd[f].fail;
        while (nd[f].child(t) < 0) {
          f = nd[f].fail;
          if (nd[f].tok == -1) break;
        }
        int c2 = nd[f].child(t);
        if (c2 >= 0) f = c2;
      }
      nd[kid].fail = f;
      int o = f;
      while (!nd[o].is_end) {
        o = nd[o].fail;
        if (nd[o].tok == -1) {
          o = -1;
          break;
        }
      }
      nd[kid].out = o;
      if (o >= 0) nd[kid].out_score += nd[o].out_score;
      q.push_back(kid);
    }
  }
  // token classes
  dfa.tok2cls.assign(V, -1);
  std::vector<int> cls_tok;
  for (size_t i = 1; i < nd.size(); ++i) {
    int t = nd[i].tok;
    if (dfa.tok2cls[t] < 0) {
      dfa.tok2cls[t] = (int)cls_tok.size();
      cls_tok.push_back(t);
    }
  }
  dfa.num_states = (int)nd.size();
  dfa.num_cls = (int)cls_tok.size();
  dfa.next.resize((size_t)dfa.num_states * dfa.num_cls);
  dfa.delta.resize((size_t)dfa.num_states * dfa.num_cls);
  dfa.node_score.resize(dfa.num_states);
  for (int s = 0; s < dfa.num_states; ++s) {
    dfa.node_score[s] = nd[s].node_score;
    for (int c = 0; c < dfa.num_cls; ++c) {
      int t = cls_tok[c];
      int n;
      double score;
      int d = nd[s].child(t);
      if (d >= 0) {
        n = d;
        score = nd[n].tok_score;
      } else {
        n = nd[s].fail;
        while (nd[n].child(t) < 0) {
          n = nd[n].fail;
          if (nd[n].tok == -1) break;
        }
        int c2 = nd[n].child(t);
        if (c2 >= 0) n = c2;
        score = nd[n].node_score - nd[s].node_score;
      }
      if (nd[n].out_score != 0) {
        double matched = nd[n].is_end ? nd[n].node_score
                                      : (nd[n].out >= 0 ? nd[nd[n].out].node_score
                                                        : nd[n].node_score);
        score = score + matched - nd[n].node_score;
        n = 0;
      }
      dfa.next[(size_t)s * dfa.num_cls + c] = n;
      dfa.delta[(size_t)s * dfa.num_cls + c] = score;
    }
  }
  return dfa;
}

// ------------------------------------------------------------------------------------
// model loading
// ------------------------------------------------------------------------------------
namespace {

ModelConfig parse_config(const std::string& text) {
  Json j = Json::parse(text);
  ModelConfig c;
  c.name = j.has("name") ? j.at("name").str : "zipformer";
  c.dims = j.at("encoder_dims").as_int_vec();
  c.layers = j.at("num_layers").as_int_vec();
  c.ff = j.at("ff_dims").as_int_vec();
  c.heads = j.at("num_heads").as_int_vec();
  c.ds = j.at("downsampling").as_int_vec();
  c.kernels = j.at("cnn_kernels").as_int_vec();
  c.qd = (int)j.at("query_head_dim").num;
  c.vd = (int)j.at("value_head_dim").num;
  c.pd = (int)j.at("pos_head_dim").num;
  c.pos_dim = (int)j.at("pos_dim").num;
  c.V = (int)j.at("vocab_size").num;
  c.dec_dim = (int)j.at("decoder_dim").num;
  c.joiner_dim = (int)j.at("joiner_dim").num;
  c.context = (int)j.at("context_size").num;
  if (j.has("layer1_channels")) c.c1 = (int)j.at("layer1_channels").num;
  if (j.has("layer2_channels")) c.c2 = (int)j.at("layer2_channels").num;
  if (j.has("layer3_channels")) c.c3 = (int)j.at("layer3_channels").num;
  ZASR_REQUIRE(c.qd == 32 && c.pd == 4, "kernels are specialised for query_head_dim 32, pos_head_dim 4");
  ZASR_REQUIRE(c.c1 == 8 && c.c2 == 32 && c.c3 == 128, "Conv2dSubsampling channels must be 8/32/128");
  ZASR_REQUIRE(c.context == 2, "decoder context_size must be 2");
  ZASR_REQUIRE(c.dec_dim == c.joiner_dim, "decoder_dim must equal joiner_dim");
  size_t ns = c.dims.size();
  ZASR_REQUIRE(c.layers.size() == ns && c.ff.size() == ns && c.heads.size() == ns &&
                   c.ds.size() == ns && c.kernels.size() == ns,
               "inconsistent stack config");
  for (size_t i = 0; i < ns; ++i) {
    ZASR_REQUIRE(c.dims[i] % 16 == 0, "encoder dims must be multiples of 16");
    ZASR_REQUIRE(c.ds[i] >= 1 && c.ds[i] <= 8, "downsampling factor must be 1..8");
  }
  return c;
}

}  // namespace

// ------------------------------------------------------------------------------------
// Engine
// ------------------------------------------------------------------------------------
template <class T>
T* Engine::ws(const std::string& name, size_t count) {
  size_t bytes = std::max<size_t>(count * sizeof(T), 256);
  Buf& b = ws_tag_.empty() ? ws_[name] : ws_[ws_tag_ + name];
  if (b.bytes < bytes) {
    if (b.p) {
      // the buffer may be in use on any of the engine's streams (encoder sets, search, copy):
      // drain the whole device before freeing it. Growth is rare (1.125x slack per buffer).
      ZASR_HIP_CHECK(hipDeviceSynchronize());
      ZASR_HIP_CHECK(hipFree(b.p));
    }
    size_t alloc = bytes + bytes / 8;
    ZASR_HIP_CHECK(hipMalloc(&b.p, alloc));
    b.bytes = alloc;
  }
  return reinterpret_cast<T*>(b.p);
}

void Engine::upload(void* dst, const void* src, size_t bytes) {
  // staged through the current pinned arena: a copy from pinned memory is truly
  // asynchronous, so enqueueing the next batch's encoder never waits for the stream (the
  // arena of a pipeline slot is reset only after that slot's previous batch has completed)
  PinArena& a = pin_[pin_cur_];
  const size_t need = (bytes + 255) & ~size_t(255);
  if (a.used + need <= a.cap) {
    char* h = a.p + a.used;
    a.used += need;
    std::memcpy(h, src, bytes);
    ZASR_HIP_CHECK(hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, st_));
    return;
  }
  a.want += need;  // grown at the arena's next reset
  // pageable source: HIP stages the copy before returning, so `src` may be reused
  ZASR_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st_));
}

void Engine::pin_reset(int arena) {
  // callers guarantee every earlier copy out of this arena has executed
  PinArena& a = pin_[arena];
  const size_t want = std::max(a.want + a.used, a.cap);
  if (want > a.cap) {
    if (a.p) ZASR_HIP_CHECK(hipHostFree(a.p));
    a.cap = want + want / 4 + 4096;
    ZASR_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&a.p), a.cap, hipHostMallocDefault));
  }
  a.used = 0;
  a.want = 0;
  pin_cur_ = arena;
}

Engine::Engine(const std::string& dir, int device, int beam, bool greedy,
               const std::vector<std::vector<int>>& hotwords, const std::vector<float>& hotword_scores,
               int precision)
    : device_(device), beam_(beam), greedy_(greedy), precision_(precision) {
  ZASR_REQUIRE(precision >= 0 && precision <= 5,
               "precision must be 0 (fp32), 1 (bf16), 2 (bf16 encoder, f32 joiner + search), 3 "
               "(bf16x3: two-piece split-bf16 products), 4 (bf16x6: three-piece, f32 quality) or "
               "5 (f16x3: fp16 hi + scaled lo pieces, f32 quality)");
  // host side first (no GPU state to unwind when the files are bad): config.json +
  // model.safetensors, or the reference's encoder-/decoder-/joiner-*.onnx (onnx_io.h;
  // core/asr_engine.py:913-928)
  SafeTensors W;
  ModelConfig cfg = parse_config(load_model_dir(dir, W));
  model_.cfg = cfg;
  hw_host_ = build_hotword_dfa(hotwords, hotword_scores, cfg.V);
  ZASR_HIP_CHECK(hipSetDevice(device_));
  // ZASR_SEARCH_CUS = N > 0: the search stream runs on CUs [0, N) and the encoder streams on
  // the rest (CU-masked queues), so the latency-bound search chain never waits for CUs held
  // by the next batch's encoder blocks
  if (const char* e = getenv("ZASR_SEARCH_CUS")) search_cus_ = atoi(e);
  int ncu = 0;
  ZASR_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_));
  if (search_cus_ > 0 && search_cus_ < ncu) {
    std::vector<uint32_t> ms((ncu + 31) / 32, 0u), me((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c) (c < search_cus_ ? ms : me)[c / 32] |= 1u << (c % 32);
    ZASR_HIP_CHECK(hipExtStreamCreateWithCUMask(&stream2_, (uint32_t)ms.size(), ms.data()));
    ZASR_HIP_CHECK(hipExtStreamCreateWithCUMask(&stream3_, (uint32_t)ms.size(), ms.data()));
    ZASR_HIP_CHECK(hipExtStreamCreateWithCUMask(&stream_, (uint32_t)me.size(), me.data()));
    for (auto& x : enc_extra_)
      ZASR_HIP_CHECK(hipExtStreamCreateWithCUMask(&x, (uint32_t)me.size(), me.data()));
  } else {
    search_cus_ = 0;
    ZASR_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    int least = 0, greatest = 0;
    ZASR_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    ZASR_HIP_CHECK(hipStreamCreateWithPriority(&stream2_, hipStreamNonBlocking, greatest));
    ZASR_HIP_CHECK(hipStreamCreateWithPriority(&stream3_, hipStreamNonBlocking, greatest));
    for (auto& x : enc_extra_) ZASR_HIP_CHECK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    // stream4_ (a third beam search in flight) is created on first use only: streams share
    // the process's hardware queues (GPU_MAX_HW_QUEUES, 4 by default) in creation order, and
    // one created ahead of the encoder streams put the second encoder stream on a shared
    // queue (greedy pipeline 107.5k -> 97.5k xRT, measured)
  }
  for (auto& e : part_ev_) ZASR_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  st_ = stream_;

  auto dev = [&](const float* src, size_t n) -> float* {
    float* p = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(float)));
    ZASR_HIP_CHECK(hipMemcpy(p, src, n * sizeof(float), hipMemcpyHostToDevice));
    model_.allocations.push_back(p);
    return p;
  };
  auto tensor = [&](const std::string& name, std::initializer_list<int64_t> shape) {
    const HostTensor& t = W.get(name);
    std::vector<int64_t> want(shape);
    ZASR_REQUIRE(t.shape == want, "shape mismatch for " + name);
    return t;
  };
  auto lin = [&](const std::string& pre, int N, int K, bool bias = true) {
    DLin l;
    l.N = N;
    l.K = K;
    const float* hw = tensor(pre + ".weight", {N, K}).data;
    if (precision_ == 5) {
      // f16x3 splits every weight into fp16 pieces: a magnitude at or beyond the fp16 range
      // would become inf, so such a model is refused here (use bf16x6: same quality)
      for (size_t i = 0; i < (size_t)N * K; ++i)
        ZASR_REQUIRE(std::fabs(hw[i]) < 65504.f,
                     "precision f16x3: weight " + pre + " exceeds the fp16 range; use bf16x6");
    }
    l.w = dev(hw, (size_t)N * K);
    if (bias) l.b = dev(tensor(pre + ".bias", {N}).data, N);
    return l;
  };
  auto vec = [&](const std::string& name, int n) { return dev(tensor(name, {n}).data, n); };
  auto scalar = [&](const std::string& name) {
    const HostTensor& t = W.get(name);
    ZASR_REQUIRE(t.numel == 1, name + " must be a scalar");
    return t.data[0];
  };

  // ---- Conv2dSubsampling ----
  {
    const HostTensor& w0 = tensor("encoder_embed.conv.0.weight", {8, 1, 3, 3});
    model_.conv0_w = dev(w0.data, 72);
    model_.conv0_b = vec("encoder_embed.conv.0.bias", 8);
    // conv.4 [32][8][3][3] -> [o][(kt*3+kf)*8 + c]
    const HostTensor& w4 = tensor("encoder_embed.conv.4.weight", {32, 8, 3, 3});
    std::vector<float> p4(32 * 72);
    for (int o = 0; o < 32; ++o)
      for (int c = 0; c < 8; ++c)
        for (int kk = 0; kk < 9; ++kk) p4[o * 72 + kk * 8 + c] = w4.data[(o * 8 + c) * 9 + kk];
    model_.conv4 = DLin{dev(p4.data(), p4.size()), vec("encoder_embed.conv.4.bias", 32), 32, 72};
    const HostTensor& w7 = tensor("encoder_embed.conv.7.weight", {128, 32, 3, 3});
    std::vector<float> p7(128 * 288);
    for (int o = 0; o < 128; ++o)
      for (int c = 0; c < 32; ++c)
        for (int kk = 0; kk < 9; ++kk) p7[o * 288 + kk * 32 + c] = w7.data[(o * 32 + c) * 9 + kk];
    model_.conv7 = DLin{dev(p7.data(), p7.size()), vec("encoder_embed.conv.7.bias", 128), 128, 288};
    model_.dw_w = dev(tensor("encoder_embed.convnext.depthwise_conv.weight", {128, 1, 7, 7}).data,
                      128 * 49);
    model_.dw_b = vec("encoder_embed.convnext.depthwise_conv.bias", 128);
    model_.pw1 = DLin{dev(tensor("encoder_embed.convnext.pointwise_conv1.weight", {384, 128, 1, 1})
                              .data, 384 * 128),
                      vec("encoder_embed.convnext.pointwise_conv1.bias", 384), 384, 128};
    model_.pw2 = DLin{dev(tensor("encoder_embed.convnext.pointwise_conv2.weight", {128, 384, 1, 1})
                              .data, 128 * 384),
                      vec("encoder_embed.convnext.pointwise_conv2.bias", 128), 128, 384};
    // out: input index c*19 + f  ->  f*128 + c  (our [L][19][128] layout)
    const int d0 = cfg.dims[0];
    const HostTensor& wo = tensor("encoder_embed.out.weight", {d0, 128 * 19});
    std::vector<float> po((size_t)d0 * 2432);
    for (int n = 0; n < d0; ++n)
      for (int c = 0; c < 128; ++c)
        for (int f = 0; f < 19; ++f) po[(size_t)n * 2432 + f * 128 + c] = wo.data[(size_t)n * 2432 + c * 19 + f];
    model_.out = DLin{dev(po.data(), po.size()), vec("encoder_embed.out.bias", d0), d0, 2432};
    model_.out_norm_b = vec("encoder_embed.out_norm.bias", d0);
    model_.out_norm_ls = scalar("encoder_embed.out_norm.log_scale");
  }
  // ---- stacks ----
  const int qd = cfg.qd, vd = cfg.vd, pd = cfg.pd;
  for (size_t i = 0; i < cfg.dims.size(); ++i) {
    DStack s;
    s.d = cfg.dims[i];
    s.F = cfg.ff[i];
    s.h = cfg.heads[i];
    s.ds = cfg.ds[i];
    s.K = cfg.kernels[i];
    const int d = s.d, F = s.F, h = s.h;
    std::string pre = "encoder.encoders." + std::to_string(i) + ".";
    if (s.ds != 1) {
      const HostTensor& b = tensor(pre + "downsample.bias", {s.ds});
      double mx = -1e30, sum = 0;
      for (int u = 0; u < s.ds; ++u) mx = std::max(mx, (double)b.data[u]);
      std::vector<double> e(s.ds);
      for (int u = 0; u < s.ds; ++u) sum += (e[u] = std::exp((double)b.data[u] - mx));
      for (int u = 0; u < s.ds; ++u) s.ds_w[u] = (float)(e[u] / sum);
      s.comb = vec(pre + "out_combiner.bypass_scale", d);
      pre += "encoder.";
    }
    for (int j = 0; j < cfg.layers[i]; ++j) {
      DLayer L;
      std::string p = pre + "layers." + std::to_string(j) + ".";
      L.bypass = vec(p + "bypass.bypass_scale", d);
      L.bypass_mid = vec(p + "bypass_mid.bypass_scale", d);
      L.attn_in = lin(p + "self_attn_weights.in_proj", (2 * qd + pd) * h, d);
      const HostTensor& pw = tensor(p + "self_attn_weights.linear_pos.weight", {pd * h, cfg.pos_dim});
      L.pos_w.assign(pw.data, pw.data + pw.numel);
      for (int a = 0; a < 2; ++a) {
        std::string n = p + "self_attn" + std::to_string(a + 1);
        L.sa_in[a] = lin(n + ".in_proj", vd * h, d);
        L.sa_out[a] = lin(n + ".out_proj", d, vd * h);
      }
      const int fdims[3] = {(F * 3) / 4, F, (F * 5) / 4};
      for (int a = 0; a < 3; ++a) {
        std::string n = p + "feed_forward" + std::to_string(a + 1);
        L.ff_in[a] = lin(n + ".in_proj", fdims[a], d);
        L.ff_out[a] = lin(n + ".out_proj", d, fdims[a]);
      }
      const int hid = 3 * d / 4;
      L.na_in = lin(p + "nonlin_attention.in_proj", 3 * hid, d);
      L.na_out = lin(p + "nonlin_attention.out_proj", d, hid);
      for (int a = 0; a < 2; ++a) {
        std::string n = p + "conv_module" + std::to_string(a + 1);
        L.cv_in[a] = lin(n + ".in_proj", 2 * d, d);
        L.cv_out[a] = lin(n + ".out_proj", d, d);
        L.cv_dw_w[a] = dev(tensor(n + ".depthwise_conv.weight", {d, 1, s.K}).data, (size_t)d * s.K);
        L.cv_dw_b[a] = vec(n + ".depthwise_conv.bias", d);
      }
      L.norm_b = vec(p + "norm.bias", d);
      L.norm_ls = scalar(p + "norm.log_scale");
      s.layers.push_back(std::move(L));
    }
    model_.stacks.push_back(std::move(s));
  }
  {
    const HostTensor& b = tensor("encoder.downsample_output.bias", {2});
    double mx = std::max(b.data[0], b.data[1]);
    double e0 = std::exp(b.data[0] - mx), e1 = std::exp(b.data[1] - mx);
    model_.out_ds_w[0] = (float)(e0 / (e0 + e1));
    model_.out_ds_w[1] = (float)(e1 / (e0 + e1));
  }
  model_.enc_proj = lin("encoder_proj", cfg.joiner_dim, cfg.max_dim());
  const int D = cfg.dec_dim;
  model_.dec_emb = dev(tensor("decoder.embedding.weight", {cfg.V, D}).data, (size_t)cfg.V * D);
  model_.dec_conv = dev(tensor("decoder.conv.weight", {D, 4, 2}).data, (size_t)D * 8);
  {
    // decoder conv taps per vocabulary entry: tap_k[v][c] = sum_ci W[c][ci][k] E[v][4(c/4)+ci]
    const HostTensor& E = tensor("decoder.embedding.weight", {cfg.V, D});
    const HostTensor& Wc = tensor("decoder.conv.weight", {D, 4, 2});
    std::vector<float> t0((size_t)cfg.V * D), t1((size_t)cfg.V * D);
    for (int v = 0; v < cfg.V; ++v)
      for (int c = 0; c < D; ++c) {
        const float* e = E.data + (size_t)v * D + (c & ~3);
        const float* w = Wc.data + (size_t)c * 8;
        float a0 = 0.f, a1 = 0.f;
        for (int ci = 0; ci < 4; ++ci) {
          a0 = std::fma(w[ci * 2 + 0], e[ci], a0);
          a1 = std::fma(w[ci * 2 + 1], e[ci], a1);
        }
        t0[(size_t)v * D + c] = a0;
        t1[(size_t)v * D + c] = a1;
      }
    model_.dec_tap0 = dev(t0.data(), t0.size());
    model_.dec_tap1 = dev(t1.data(), t1.size());
  }
  model_.dec_proj = lin("decoder_proj", cfg.joiner_dim, D);
  model_.joiner = lin("joiner.output_linear", cfg.V, cfg.joiner_dim);
  ensure_pos_tables(2048);
  // the conv modules' in_proj: rows interleaved (a_c, s_c) for the GLU epilogue (EPI_GLU)
  auto glu_interleave = [&](DLin& l) {
    const int d = l.N / 2, K = l.K;
    std::vector<float> w((size_t)l.N * K), wi((size_t)l.N * K), b(l.N), bi(l.N);
    ZASR_HIP_CHECK(hipMemcpy(w.data(), l.w, w.size() * 4, hipMemcpyDeviceToHost));
    if (l.b) ZASR_HIP_CHECK(hipMemcpy(b.data(), l.b, b.size() * 4, hipMemcpyDeviceToHost));
    for (int c = 0; c < d; ++c)
      for (int h = 0; h < 2; ++h) {
        std::memcpy(&wi[(size_t)(2 * c + h) * K], &w[(size_t)(h * d + c) * K], (size_t)K * 4);
        bi[2 * c + h] = b[h * d + c];
      }
    float* pw = dev(wi.data(), wi.size());
    float* pb = l.b ? dev(bi.data(), bi.size()) : nullptr;
    l.w = pw;
    l.b = pb;
    l.glu = true;
  };
  if (split_pieces() > 0) {  // split-bf16 pieces of every encoder projection weight
    auto mkx = [&](DLin& l) {
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, (size_t)l.N * l.K * 2 * stored_pieces(split_pieces())));
      model_.allocations.push_back(p);
      split_to_bf16(l.w, p, (long)l.N * l.K, split_pieces(), stream_);
      l.wx = p;
    };
    for (DLin* l : {&model_.conv4, &model_.conv7, &model_.pw1, &model_.pw2, &model_.out,
                    &model_.enc_proj, &model_.joiner})
      mkx(*l);
    if (split_pieces() == kPiecesF16) {
      // the fused f16x3 ConvNeXt MLP reads pw1 / pw2 as fp16 piece images in MFMA-fragment
      // order (pack_frag32_host per piece, the same split as split_to_bf16)
      for (DLin* l : {&model_.pw1, &model_.pw2}) {
        const size_t n = (size_t)l->N * l->K;
        std::vector<float> w(n);
        ZASR_HIP_CHECK(hipMemcpy(w.data(), l->w, n * 4, hipMemcpyDeviceToHost));
        std::vector<__bf16> piece(n), pk(2 * n);
        for (int t = 0; t < 2; ++t) {
          for (size_t i = 0; i < n; ++i) {
            const _Float16 hi = (_Float16)w[i];
            const _Float16 v = t == 0 ? hi : (_Float16)((w[i] - (float)hi) * 2048.f);
            std::memcpy(&piece[i], &v, 2);
          }
          pack_frag32_host(piece.data(), l->N, l->K, pk.data() + t * n);
        }
        void* p = nullptr;
        ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
        model_.allocations.push_back(p);
        ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
        l->wp = p;
      }
    }
    if (split_pieces() == kPiecesF16) {
      // the fused f16x3 FFN (model dims 256..512) reads W1 / W2 as fp16 piece images in
      // MFMA-fragment order; a layer whose weights reach 31 in magnitude keeps the GEMM pair
      for (auto& s : model_.stacks)
        for (auto& L : s.layers)
          for (int a = 0; a < 3; ++a) {
            const int F = L.ff_in[a].N, d = L.ff_in[a].K;
            if (!ffn_h3_supported(d, F)) continue;
            std::vector<float> w1((size_t)F * d), w2((size_t)F * d);
            ZASR_HIP_CHECK(hipMemcpy(w1.data(), L.ff_in[a].w, w1.size() * 4, hipMemcpyDeviceToHost));
            ZASR_HIP_CHECK(hipMemcpy(w2.data(), L.ff_out[a].w, w2.size() * 4, hipMemcpyDeviceToHost));
            if (!ffn_h3_weights_ok(w1.data(), (long)w1.size()) || !ffn_h3_weights_ok(w2.data(), (long)w2.size())) {
              ++routes_.ffn_gemm_pair;
              continue;
            }
            ++routes_.ffn_fused_h3;
            for (auto [l, w] : {std::pair<DLin*, std::vector<float>*>{&L.ff_in[a], &w1},
                                std::pair<DLin*, std::vector<float>*>{&L.ff_out[a], &w2}}) {
              std::vector<__bf16> pk(2 * w->size());
              ffn_pack_h3_host(w->data(), l->N, l->K, pk.data());
              void* p = nullptr;
              ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
              model_.allocations.push_back(p);
              ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
              l->wp = p;
            }
          }
    }
    if (cfg.joiner_dim == 256 || cfg.joiner_dim == 512) {
      // the joiner's W pieces in MFMA-fragment order (one packed image per piece) for
      // joiner_split_packed_kernel; J is written in the same order, already split, by store_j4
      const long pe = gemm_rp_packed_elems(cfg.V, cfg.joiner_dim);
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, (size_t)pe * 2 * stored_pieces(split_pieces())));
      model_.allocations.push_back(p);
      for (int t = 0; t < stored_pieces(split_pieces()); ++t)
        gemm_rp_pack_weights(reinterpret_cast<const __bf16*>(model_.joiner.wx) + (long)t * cfg.V * cfg.joiner_dim,
                             cfg.V, cfg.joiner_dim, reinterpret_cast<__bf16*>(p) + t * pe, stream_);
      model_.joiner_packed = p;
      model_.joiner_plane = pe;
    }
    for (auto& s : model_.stacks)
      for (auto& L : s.layers) {
        for (int a = 0; a < 2; ++a) glu_interleave(L.cv_in[a]);
        for (DLin* l : {&L.attn_in, &L.na_in, &L.na_out}) mkx(*l);
        for (int a = 0; a < 2; ++a)
          for (DLin* l : {&L.sa_in[a], &L.sa_out[a], &L.cv_in[a], &L.cv_out[a]}) mkx(*l);
        for (int a = 0; a < 3; ++a)
          for (DLin* l : {&L.ff_in[a], &L.ff_out[a]}) mkx(*l);
      }
    ZASR_HIP_CHECK(hipStreamSynchronize(stream_));
    if (split_pieces() == kPiecesF16) {
      // the layer projections the row-resident f16x3 GEMM takes (K, N within its shapes and
      // every |w| < 31; the others keep gemm_x3)
      auto mkr = [&](DLin& l) {
        if (!gemm_h3r_supported(l.K, l.N, EPI_NONE)) return;
        std::vector<float> w((size_t)l.N * l.K);
        ZASR_HIP_CHECK(hipMemcpy(w.data(), l.w, w.size() * 4, hipMemcpyDeviceToHost));
        if (!ffn_h3_weights_ok(w.data(), (long)w.size())) {
          ++routes_.gemm_x3_range;
          return;
        }
        ++routes_.gemm_h3r;
        std::vector<__bf16> pk(2 * w.size());
        ffn_pack_h3_host(w.data(), l.N, l.K, pk.data());
        void* p = nullptr;
        ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
        model_.allocations.push_back(p);
        ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
        l.wr = p;
      };
      for (auto& s : model_.stacks)
        for (auto& L : s.layers) {
          for (DLin* l : {&L.attn_in, &L.na_in, &L.na_out}) mkr(*l);
          for (int a = 0; a < 2; ++a)
            for (DLin* l : {&L.sa_in[a], &L.sa_out[a], &L.cv_in[a], &L.cv_out[a]}) mkr(*l);
        }
      // the ConvNeXt MLP (pw1 [384][128], pw2 [128][384]) as the fused f16x3 FFN
      if (model_.pw1.K == 128 && model_.pw2.N == 128 && ffn_h3_supported(128, model_.pw1.N)) {
        std::vector<float> w1((size_t)model_.pw1.N * 128), w2(w1.size());
        ZASR_HIP_CHECK(hipMemcpy(w1.data(), model_.pw1.w, w1.size() * 4, hipMemcpyDeviceToHost));
        ZASR_HIP_CHECK(hipMemcpy(w2.data(), model_.pw2.w, w2.size() * 4, hipMemcpyDeviceToHost));
        const bool ok = ffn_h3_weights_ok(w1.data(), (long)w1.size()) && ffn_h3_weights_ok(w2.data(), (long)w2.size());
        routes_.cnx_ffn_h3 = ok ? 1 : 0;
        if (ok)
          for (auto [l, w] : {std::pair<DLin*, std::vector<float>*>{&model_.pw1, &w1},
                              std::pair<DLin*, std::vector<float>*>{&model_.pw2, &w2}}) {
            std::vector<__bf16> pk(2 * w->size());
            ffn_pack_h3_host(w->data(), l->N, l->K, pk.data());
            void* p = nullptr;
            ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
            model_.allocations.push_back(p);
            ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
            l->wr = p;
          }
      }
    }
  }
  if (precision_ == 1 || precision_ == 2) {  // bf16 copies of every dense projection weight
    for (auto& s : model_.stacks)
      for (auto& L : s.layers)
        for (int a = 0; a < 2; ++a) glu_interleave(L.cv_in[a]);
    auto mk = [&](DLin& l) {
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, (size_t)l.N * l.K * 2));
      model_.allocations.push_back(p);
      convert_to_bf16(l.w, p, (long)l.N * l.K, stream_);
      l.wh = p;
    };
    for (DLin* l : {&model_.conv4, &model_.conv7, &model_.pw1, &model_.pw2, &model_.out,
                    &model_.enc_proj})
      mk(*l);
    // precision 2 keeps the joiner (and with it J, the logits and the search) in f32
    if (precision_ == 1) mk(model_.joiner);
    if (precision_ == 1 && (cfg.joiner_dim == 256 || cfg.joiner_dim == 512)) {  // speculative-greedy joiner operand
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, (size_t)gemm_rp_packed_elems(cfg.V, cfg.joiner_dim) * 2));
      model_.allocations.push_back(p);
      gemm_rp_pack_weights(model_.joiner.wh, cfg.V, cfg.joiner_dim, p, stream_);
      model_.joiner_packed = p;
    }
    for (auto& s : model_.stacks)
      for (auto& L : s.layers) {
        // attn_in: the query and positional-query rows carry log2(e) in the bf16 path (the
        // flash attention works in the log2 domain), folded before the single rounding
        {
          DLin& l = L.attn_in;
          const int h = s.h;
          std::vector<float> rs(l.N, 1.f), bias(l.N);
          const float kLog2e = 1.4426950408889634f;
          for (int r = 0; r < l.N; ++r)
            if (r < 32 * h || r >= 64 * h) rs[r] = kLog2e;
          ZASR_HIP_CHECK(hipMemcpy(bias.data(), l.b, l.N * sizeof(float), hipMemcpyDeviceToHost));
          for (int r = 0; r < l.N; ++r) bias[r] *= rs[r];
          float* d_rs = dev(rs.data(), rs.size());
          l.bh = dev(bias.data(), bias.size());
          void* p = nullptr;
          ZASR_HIP_CHECK(hipMalloc(&p, (size_t)l.N * l.K * 2));
          model_.allocations.push_back(p);
          convert_rows_to_bf16(l.w, d_rs, p, l.N, l.K, stream_);
          l.wh = p;
        }
        for (DLin* l : {&L.na_in, &L.na_out}) mk(*l);
        for (int a = 0; a < 2; ++a)
          for (DLin* l : {&L.sa_in[a], &L.sa_out[a], &L.cv_in[a], &L.cv_out[a]}) mk(*l);
        for (int a = 0; a < 3; ++a)
          for (DLin* l : {&L.ff_in[a], &L.ff_out[a]}) mk(*l);
      }
    ZASR_HIP_CHECK(hipStreamSynchronize(stream_));
    // the ConvNeXt MLP reads pw1 / pw2 in MFMA-fragment order
    for (DLin* l : {&model_.pw1, &model_.pw2}) {
      std::vector<__bf16> h((size_t)l->N * l->K), pk(h.size());
      ZASR_HIP_CHECK(hipMemcpy(h.data(), l->wh, h.size() * 2, hipMemcpyDeviceToHost));
      pack_frag32_host(h.data(), l->N, l->K, pk.data());
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
      model_.allocations.push_back(p);
      ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
      l->wp = p;
    }
    // the wide fused FFN (model dims 256..512) reads W1 / W2 in MFMA-fragment order
    for (auto& s : model_.stacks)
      for (auto& L : s.layers)
        for (int a = 0; a < 3; ++a) {
          const int F = L.ff_in[a].N, d = L.ff_in[a].K;
          if (d < 256 || !ffn_fused_supported(d) || F % 32 != 0 || F > 2048) continue;
          for (DLin* l : {&L.ff_in[a], &L.ff_out[a]}) {
            std::vector<__bf16> h((size_t)l->N * l->K), pk(h.size());
            ZASR_HIP_CHECK(hipMemcpy(h.data(), l->wh, h.size() * 2, hipMemcpyDeviceToHost));
            ffn_pack_host(h.data(), l->N, l->K, pk.data());
            void* p = nullptr;
            ZASR_HIP_CHECK(hipMalloc(&p, pk.size() * 2));
            model_.allocations.push_back(p);
            ZASR_HIP_CHECK(hipMemcpy(p, pk.data(), pk.size() * 2, hipMemcpyHostToDevice));
            l->wp = p;
          }
        }
  }
  // ---- decoder-context table (kernels.h, DecTable): V^2 x D f32, built once ----
  {
    const double gb = (double)cfg.V * cfg.V * cfg.joiner_dim * 4.0 / 1e9;
    double max_gb = 24.0;
    if (const char* e = getenv("ZASR_DEC_TABLE_MAX_GB")) max_gb = atof(e);
    if (gb <= max_gb) {
      void* p = nullptr;
      ZASR_HIP_CHECK(hipMalloc(&p, (size_t)cfg.V * cfg.V * cfg.joiner_dim * sizeof(float)));
      model_.allocations.push_back(p);
      model_.dec_table = reinterpret_cast<float*>(p);
      DecoderW dw{model_.dec_tap0, model_.dec_tap1, model_.dec_proj.b, cfg.joiner_dim};
      launch_dec_table(dw, model_.dec_proj.w, cfg.V, model_.dec_table, stream_);
      ZASR_HIP_CHECK(hipStreamSynchronize(stream_));
    }
  }

  // ---- fbank tables ----
  {
    std::vector<double> tw(512);
    for (int j = 0; j < 256; ++j) {
      double a = -2.0 * M_PI * j / 512.0;
      tw[2 * j] = std::cos(a);
      tw[2 * j + 1] = std::sin(a);
    }
    ZASR_HIP_CHECK(hipMalloc(&d_twiddle_, 512 * sizeof(double)));
    ZASR_HIP_CHECK(hipMemcpy(d_twiddle_, tw.data(), 512 * sizeof(double), hipMemcpyHostToDevice));
    std::vector<float> win(400);
    for (int i = 0; i < 400; ++i)
      win[i] = (float)std::pow(0.5 - 0.5 * std::cos(2.0 * M_PI / 399.0 * i), 0.85);
    d_window_ = dev(win.data(), 400);
    // knf's triangles: mel-linear between 20 Hz and 7600 Hz over the bins 0 .. 255
    auto mel = [](float f) { return 1127.0f * logf(1.0f + f / 700.0f); };
    const float mlo = mel(20.0f), mhi = mel(7600.0f);
    const float delta = (mhi - mlo) / 81.0f;
    std::vector<float> banks(80 * 256, 0.f);
    for (int b = 0; b < 80; ++b) {
      float left = mlo + (float)b * delta, center = mlo + (float)(b + 1) * delta,
            right = mlo + (float)(b + 2) * delta;
      for (int i = 0; i < 256; ++i) {
        float m = mel(31.25f * (float)i);
        if (m > left && m < right)
          banks[b * 256 + i] = (m <= center) ? (m - left) / (center - left) : (right - m) / (right - center);
      }
    }
    set_mel_banks(banks.data(), 256);
  }
  // ---- hotwords ----
  hw_.num_states = hw_host_.num_states;
  hw_.num_cls = hw_host_.num_cls;
  if (hw_host_.num_states > 0) {
    int *t2c = nullptr, *nx = nullptr;
    double *dl = nullptr, *ns = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&t2c, hw_host_.tok2cls.size() * sizeof(int)));
    ZASR_HIP_CHECK(hipMalloc(&nx, std::max<size_t>(hw_host_.next.size(), 1) * sizeof(int)));
    ZASR_HIP_CHECK(hipMalloc(&dl, std::max<size_t>(hw_host_.delta.size(), 1) * sizeof(double)));
    ZASR_HIP_CHECK(hipMalloc(&ns, hw_host_.node_score.size() * sizeof(double)));
    ZASR_HIP_CHECK(hipMemcpy(t2c, hw_host_.tok2cls.data(), hw_host_.tok2cls.size() * sizeof(int), hipMemcpyHostToDevice));
    ZASR_HIP_CHECK(hipMemcpy(nx, hw_host_.next.data(), hw_host_.next.size() * sizeof(int), hipMemcpyHostToDevice));
    ZASR_HIP_CHECK(hipMemcpy(dl, hw_host_.delta.data(), hw_host_.delta.size() * sizeof(double), hipMemcpyHostToDevice));
    ZASR_HIP_CHECK(hipMemcpy(ns, hw_host_.node_score.data(), hw_host_.node_score.size() * sizeof(double), hipMemcpyHostToDevice));
    model_.allocations.push_back(t2c);
    model_.allocations.push_back(nx);
    model_.allocations.push_back(dl);
    model_.allocations.push_back(ns);
    hw_.tok2cls = t2c;
    hw_.next = nx;
    hw_.delta = dl;
    hw_.node_score = ns;
  }
  ZASR_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_pinned_), 64, hipHostMallocDefault));
  ZASR_HIP_CHECK(hipDeviceSynchronize());
}

void Engine::set_mel_banks(const float* banks, int n_bins) {
  ZASR_REQUIRE(n_bins == 256 || n_bins == 257, "mel banks: 256 or 257 bins per filter");
  // sparse rows: first nonzero bin, run length, offset into the packed weights
  std::vector<int> meta(240);
  std::vector<float> wts;
  for (int b = 0; b < 80; ++b) {
    const float* row = banks + (size_t)b * n_bins;
    if (n_bins == 257)
      ZASR_REQUIRE(row[256] == 0.f, "mel banks: the Nyquist bin must carry no weight");
    int st = -1, en = -1;
    for (int i = 0; i < 256; ++i)
      if (row[i] != 0.f) {
        if (st < 0) st = i;
        en = i;
      }
    if (st < 0) st = en = 0;
    meta[b] = st;
    meta[80 + b] = en - st + 1;
    meta[160 + b] = (int)wts.size();
    for (int i = st; i <= en; ++i) wts.push_back(row[i]);
  }
  ZASR_HIP_CHECK(hipDeviceSynchronize());  // no fbank in flight reads the old tables
  if (!d_mel_meta_) ZASR_HIP_CHECK(hipMalloc(&d_mel_meta_, 240 * sizeof(int)));
  ZASR_HIP_CHECK(hipMemcpy(d_mel_meta_, meta.data(), 240 * sizeof(int), hipMemcpyHostToDevice));
  if (d_mel_w_) ZASR_HIP_CHECK(hipFree(d_mel_w_));
  d_mel_w_ = nullptr;
  ZASR_HIP_CHECK(hipMalloc(&d_mel_w_, wts.size() * sizeof(float)));
  ZASR_HIP_CHECK(hipMemcpy(d_mel_w_, wts.data(), wts.size() * sizeof(float), hipMemcpyHostToDevice));
}

std::string Engine::routes_json() const {
  std::ostringstream os;
  os << "{\"precision\": " << precision_ << ", \"ffn_fused_h3\": " << routes_.ffn_fused_h3
     << ", \"ffn_gemm_pair\": " << routes_.ffn_gemm_pair << ", \"gemm_h3r\": " << routes_.gemm_h3r
     << ", \"gemm_x3_range\": " << routes_.gemm_x3_range << ", \"cnx_ffn_h3\": " << routes_.cnx_ffn_h3
     << ", \"dec_table\": " << (model_.dec_table ? 1 : 0) << "}";
  return os.str();
}

Engine::~Engine() {
  // best-effort teardown: errors here cannot be reported to the caller
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  for (void* p : model_.allocations) (void)hipFree(p);
  for (auto& s : model_.stacks)
    for (auto& l : s.layers)
      if (l.pos_tab) (void)hipFree(l.pos_tab);
  for (auto& kv : ws_)
    if (kv.second.p) (void)hipFree(kv.second.p);
  if (d_twiddle_) (void)hipFree(d_twiddle_);
  if (d_mel_meta_) (void)hipFree(d_mel_meta_);
  if (d_mel_w_) (void)hipFree(d_mel_w_);
  for (auto e : event_pool_) (void)hipEventDestroy(e);
  for (auto& pe : prof_pending_) {
    (void)hipEventDestroy(pe.a);
    (void)hipEventDestroy(pe.b);
  }
  if (copy_st_) (void)hipStreamSynchronize(copy_st_);
  for (auto e : upload_ev_)
    if (e) (void)hipEventDestroy(e);
  if (copy_st_) (void)hipStreamDestroy(copy_st_);
  (void)hipStreamSynchronize(stream2_);
  (void)hipStreamSynchronize(stream3_);
  if (stream4_) (void)hipStreamSynchronize(stream4_);
  if (h_pinned_) (void)hipHostFree(h_pinned_);
  for (auto& r : res_pin_)
    if (r.p) (void)hipHostFree(r.p);
  for (auto& a : pin_)
    if (a.p) (void)hipHostFree(a.p);
  for (auto e : part_ev_) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(stream2_);
  (void)hipStreamDestroy(stream3_);
  if (stream4_) (void)hipStreamDestroy(stream4_);
  for (auto x : enc_extra_) {
    (void)hipStreamSynchronize(x);
    (void)hipStreamDestroy(x);
  }
  (void)hipStreamDestroy(stream_);
}

// CompactRelPositionalEncoding (icefall zipformer.py, 3P) folded through linear_pos:
// table[x + pmax - 1][n] = sum_c W_pos[n][c] * pe(x)[c]
void Engine::ensure_pos_tables(int need) {
  if (need <= model_.pmax) return;
  // the tables are shared by every encoder stream: replace them only on an idle device
  ZASR_HIP_CHECK(hipDeviceSynchronize());
  int pmax = 1024;
  while (pmax < need) pmax *= 2;
  const int P = model_.cfg.pos_dim;
  const int rows = 2 * pmax - 1;
  std::vector<double> pe((size_t)rows * P);
  const double cl = std::sqrt((double)P);
  const double ls = P / (2.0 * M_PI);
  for (int r = 0; r < rows; ++r) {
    double x = (double)(r - (pmax - 1));
    double sgn = (x > 0) - (x < 0);
    double xc = cl * sgn * (std::log(std::fabs(x) + cl) - std::log(cl));
    double xa = std::atan(xc / ls);
    for (int i = 0; i < P / 2; ++i) {
      pe[(size_t)r * P + 2 * i] = std::cos(xa * (i + 1));
      pe[(size_t)r * P + 2 * i + 1] = std::sin(xa * (i + 1));
    }
    pe[(size_t)r * P + P - 1] = 1.0;
  }
  for (auto& s : model_.stacks) {
    const int n4 = 4 * s.h;
    for (auto& l : s.layers) {
      std::vector<float> tab((size_t)rows * n4);
      for (int r = 0; r < rows; ++r)
        for (int n = 0; n < n4; ++n) {
          double acc = 0;
          const double* pr = &pe[(size_t)r * P];
          const float* wr = &l.pos_w[(size_t)n * P];
          for (int c = 0; c < P; ++c) acc += (double)wr[c] * pr[c];
          tab[(size_t)r * n4 + n] = (float)acc;
        }
      if (l.pos_tab) {
        ZASR_HIP_CHECK(hipStreamSynchronize(st_));
        ZASR_HIP_CHECK(hipFree(l.pos_tab));
      }
      ZASR_HIP_CHECK(hipMalloc(&l.pos_tab, tab.size() * sizeof(float)));
      ZASR_HIP_CHECK(hipMemcpy(l.pos_tab, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice));
    }
  }
  model_.pmax = pmax;
}

// ------------------------------------------------------------------------------------
// profiling
// ------------------------------------------------------------------------------------
hipEvent_t Engine::take_event() {
  if (!event_pool_.empty()) {
    hipEvent_t e = event_pool_.back();
    event_pool_.pop_back();
    return e;
  }
  hipEvent_t e;
  ZASR_HIP_CHECK(hipEventCreate(&e));
  return e;
}

void Engine::prof_begin(const char* name) { prof_begin(std::string(name)); }

void Engine::prof_begin(const std::string& name) {
  if (!prof_on_) return;
  ProfEvent pe{name, take_event(), take_event()};
  ZASR_HIP_CHECK(hipEventRecord(pe.a, st_));
  prof_pending_.push_back(pe);
}

void Engine::prof_end() {
  if (!prof_on_ || prof_pending_.empty()) return;
  ZASR_HIP_CHECK(hipEventRecord(prof_pending_.back().b, st_));
}

void Engine::profile_reset() {
  prof_acc_.clear();
  for (auto& pe : prof_pending_) {
    event_pool_.push_back(pe.a);
    event_pool_.push_back(pe.b);
  }
  prof_pending_.clear();
}

std::string Engine::profile_report() {
  for (auto& pe : prof_pending_) {
    ZASR_HIP_CHECK(hipEventSynchronize(pe.b));
    float ms = 0.f;
    ZASR_HIP_CHECK(hipEventElapsedTime(&ms, pe.a, pe.b));
    auto& acc = prof_acc_[pe.name];
    acc.first += 1;
    acc.second += ms;
    event_pool_.push_back(pe.a);
    event_pool_.push_back(pe.b);
  }
  prof_pending_.clear();
  std::ostringstream os;
  for (auto& kv : prof_acc_) os << kv.first << " " << kv.second.first << " " << kv.second.second << "\n";
  return os.str();
}

// per-shape GEMM class names (profile mode 2): "<class>|M|K|N|w16|a16|c16|epi", parsed by
// bench.py into the per-shape roofline table
std::string Engine::shape_key(const char* cls, int M, int K, int N, bool w16, bool a16, bool c16,
                              int epi) {
  std::ostringstream os;
  os << cls << "|" << M << "|" << K << "|" << N << "|" << (int)w16 << "|" << (int)a16 << "|"
     << (int)c16 << "|" << epi;
  return os.str();
}

// ------------------------------------------------------------------------------------
// building blocks
// ------------------------------------------------------------------------------------
void Engine::linear(const DLin& l, const float* A, int lda, int M, float* C, int ldc, int epi,
                    const char* cls, const float* byp_orig, const float* byp_scale) {
  GemmParams p{};
  p.A = A;
  p.lda = lda;
  p.B = l.w;
  p.sbk = 1;
  p.sbn = l.K;
  p.C = C;
  p.ldc = ldc;
  p.bias = l.b;
  p.M = M;
  p.N = l.N;
  p.K = l.K;
  p.alpha = 1.f;
  p.max_M = M;
  ZASR_REQUIRE(byp_orig == nullptr || l.wx, "bypass epilogue: split-mode weights only");
  p.byp_orig = byp_orig;
  p.byp_scale = byp_scale;
  if (prof_shapes_ && prof_on_)
    prof_begin(shape_key(cls, M, l.K, l.N, l.wh != nullptr, false, false, epi));
  else
    prof_begin(cls);
  if (l.wr && lda == l.K && byp_orig == nullptr && gemm_h3r_supported(l.K, l.N, epi))
    gemm_h3r(A, l.wr, l.b, C, ldc, M, l.N, l.K, epi, st_);
  else if (l.wx)
    gemm_x3(p, l.wx, (long)l.N * l.K, epi, ALOAD_DENSE, st_, split_pieces());
  else if (l.wh)
    gemm_bf16(p, l.wh, epi, ALOAD_DENSE, st_);
  else
    gemm_f32(p, epi, ALOAD_DENSE, false, st_);
  prof_end();
}

void Engine::linear_h(const DLin& l, const void* A, bool a_bf16, int lda, int M, void* C,
                      bool c_bf16, int ldc, int epi, const float* byp_orig,
                      const float* byp_scale) {
  ZASR_REQUIRE(l.wh != nullptr, "linear_h needs bf16 weights");
  GemmParams p{};
  p.A = reinterpret_cast<const float*>(A);
  p.lda = lda;
  p.B = l.w;
  p.sbk = 1;
  p.sbn = l.K;
  p.C = reinterpret_cast<float*>(C);
  p.ldc = ldc;
  p.bias = l.bh ? l.bh : l.b;
  p.M = M;
  p.N = l.N;
  p.K = l.K;
  p.alpha = 1.f;
  p.max_M = M;
  p.byp_orig = byp_orig;
  p.byp_scale = byp_scale;
  if (prof_shapes_ && prof_on_)
    prof_begin(shape_key("enc_gemm", M, l.K, l.N, true, a_bf16, c_bf16, epi));
  else
    prof_begin("enc_gemm");
  gemm_bf16(p, l.wh, epi, ALOAD_DENSE, st_, a_bf16, c_bf16);
  prof_end();
}

void Engine::run_fbank(const float* d_wav, const std::vector<long>& wav_off,
                       const std::vector<long>& n, float* d_feats, std::vector<int>& frames) {
  const int B = (int)n.size();
  std::vector<long> off(B);
  std::vector<int> ns(B), fo(B + 1, 0);
  frames.resize(B);
  for (int b = 0; b < B; ++b) {
    off[b] = wav_off[b];
    ns[b] = (int)n[b];
    frames[b] = n[b] > 0 ? (int)((n[b] + 80) / 160) : 0;
    fo[b + 1] = fo[b] + frames[b];
  }
  long* d_off = ws<long>("fb_wavoff", B);
  int* d_meta = ws<int>("fb_meta", 2 * B + 1);
  std::vector<int> meta(ns);
  meta.insert(meta.end(), fo.begin(), fo.end());
  upload(d_off, off.data(), B * sizeof(long));
  upload(d_meta, meta.data(), meta.size() * sizeof(int));
  FbankTables t{d_twiddle_, d_window_, d_mel_meta_, d_mel_meta_ + 80, d_mel_meta_ + 160, d_mel_w_};
  prof_begin("fbank");
  launch_fbank(d_wav, d_off, d_meta, d_meta + B, B, fo[B], t, d_feats, st_);
  prof_end();
}

namespace {
struct LevelMeta {
  std::vector<int> len;  // per sequence
  std::vector<int> off;  // B + 1
  int total = 0, maxlen = 0;
};
LevelMeta make_level(const std::vector<int>& len) {
  LevelMeta m;
  m.len = len;
  m.off.assign(len.size() + 1, 0);
  for (size_t b = 0; b < len.size(); ++b) {
    m.off[b + 1] = m.off[b] + len[b];
    m.maxlen = std::max(m.maxlen, len[b]);
  }
  m.total = m.off.back();
  return m;
}
struct MetaPack {
  std::vector<char> bytes;
  size_t add(const void* p, size_t n) {
    size_t at = (bytes.size() + 15) & ~size_t(15);
    bytes.resize(at + n);
    if (n) std::memcpy(bytes.data() + at, p, n);
    return at;
  }
};
}  // namespace

void Engine::layer_forward(const DStack& S, const DLayer& Ly, float* X, int R, const int* d_off,
                           const int* d_map,
                           const std::vector<int>& lens, const long* d_aoff,
                           const void* d_slices_nl, int maxL, const int* d_o8, int R8, bool orig_ready, bool last_layer) {
  const int d = S.d, h = S.h, B = (int)lens.size();
  const int hid = 3 * d / 4;
  float* O = ws<float>("ly_orig", (size_t)R * d);
  if (!orig_ready)  // else the previous layer's BiasNorm already wrote src here
    ZASR_HIP_CHECK(hipMemcpyAsync(O, X, (size_t)R * d * sizeof(float), hipMemcpyDeviceToDevice, st_));
  // attention weights (shared by nonlin_attention, self_attn1, self_attn2)
  const bool bf16 = precision_ == 1 || precision_ == 2;
  const int np = split_pieces();
  float* qkp = nullptr;
  float* A = nullptr;
  __bf16* A16 = nullptr;
  float* stats = nullptr;
  AttnFlashArgs fa{};
  if (bf16) {
    // flash-style attention on bf16 q / k / v (attn_kernels.hip): head 0's normalised weights
    // for the NonlinAttention GEMM; every head's statistics come from self_attn1
    __bf16* qkp16 = ws<__bf16>("ly_qkp_h", (size_t)R * 68 * h);
    linear_h(Ly.attn_in, X, false, d, R, qkp16, true, 68 * h, EPI_NONE);
    A16 = ws<__bf16>("ly_attn_h", 1);  // sized by the caller
    stats = ws<float>("ly_attn_stats", (size_t)R * h);
    fa = AttnFlashArgs{qkp16, h, Ly.pos_tab, model_.pmax, d_off, d_aoff, B, maxL, A16,
                       nullptr, nullptr, stats, stats};
    // (head 0's weights are consumed inside the fused NonlinAttention kernel, mode 3)
  } else if (np) {
    // split-bf16 modes: the same flash kernels on f32 q / k / v, every MFMA product split
    // into np bf16 pieces per operand; head 0's weights in f32 (L8 row stride)
    qkp = ws<float>("ly_qkp", (size_t)R * 68 * h);
    linear(Ly.attn_in, X, d, R, qkp, 68 * h, EPI_NONE);
    A = ws<float>("ly_attn", 1);  // sized by the caller
    stats = ws<float>("ly_attn_stats", (size_t)R * h);
    fa = AttnFlashArgs{qkp, h, Ly.pos_tab, model_.pmax, d_off, d_aoff, B, maxL, A,
                       nullptr, nullptr, stats, stats, np};
    if (np != kPiecesF16) {  // f16x3: consumed in the fused NonlinAttention kernel
      prof_begin("attn_softmax");
      launch_attn_flash(fa, 0, st_);
      prof_end();
    }
  } else {
    // head 0 only: its normalised weights feed nonlin_attention; every head's statistics
    // come from self_attn1's online softmax
    qkp = ws<float>("ly_qkp", (size_t)R * 68 * h);
    linear(Ly.attn_in, X, d, R, qkp, 68 * h, EPI_NONE);
    A = ws<float>("ly_attn", 1);  // sized by the caller
    stats = ws<float>("ly_attn_stats", (size_t)R * h * 2);
    AttnArgs a{qkp, h, Ly.pos_tab, model_.pmax, d_off, d_aoff, B, maxL, A, stats, 1};
    prof_begin("attn_softmax");
    launch_attn_softmax(a, st_);
    prof_end();
  }
  // bf16 mode: feed_forward2's residual epilogue also applies bypass_mid (same formula as
  // launch_bypass, one pass over X fewer)
  auto ff = [&](int k) {
    const DLin& fi = Ly.ff_in[k];
    const float* bo = (bf16 && k == 1) ? O : nullptr;
    const float* bs = (bf16 && k == 1) ? Ly.bypass_mid : nullptr;
    if (fi.wh && ffn_fused_supported(d) && (d < 256 || fi.wp)) {
      // bf16 mode: in_proj -> SwooshL -> out_proj + residual in one kernel, hidden on chip
      // (d >= 256: the fragment-packed weights of ffn_wide_kernel)
      prof_begin("ffn_fused");
      launch_ffn_fused(X, R, d, fi.N, d < 256 ? fi.wh : fi.wp, fi.b,
                       d < 256 ? Ly.ff_out[k].wh : Ly.ff_out[k].wp, Ly.ff_out[k].b, st_, bo, bs);
      prof_end();
      return;
    }
    if (fi.wh) {  // bf16 mode: the hidden activation crosses HBM in bf16
      __bf16* H = ws<__bf16>("ly_hid_h", (size_t)R * fi.N);
      linear_h(fi, X, false, d, R, H, true, fi.N, EPI_SWOOSHL);
      linear_h(Ly.ff_out[k], H, true, fi.N, R, X, false, d, EPI_RESADD, bo, bs);
    } else if (fi.wp && np == kPiecesF16) {
      // f16x3 mode: the same fusion at f32 quality, the hidden layer on chip as fp16 pieces;
      // feed_forward2 folds bypass_mid as the GEMM pair's residual epilogue does
      prof_begin("ffn_fused");
      launch_ffn_fused_h3(X, R, d, fi.N, fi.wp, fi.b, Ly.ff_out[k].wp, Ly.ff_out[k].b, st_,
                          k == 1 ? O : nullptr, k == 1 ? Ly.bypass_mid : nullptr);
      prof_end();
    } else {
      // split modes: feed_forward2's epilogue applies bypass_mid too (fp32: launch_bypass)
      const bool byp = k == 1 && Ly.ff_out[k].wx != nullptr;
      float* H = ws<float>("ly_hid", (size_t)R * fi.N);
      linear(fi, X, d, R, H, fi.N, EPI_SWOOSHL);
      linear(Ly.ff_out[k], H, fi.N, R, X, d, EPI_RESADD, "enc_gemm", byp ? O : nullptr,
             byp ? Ly.bypass_mid : nullptr);
    }
  };
  auto self_attn = [&](int k) {
    if (bf16) {
      __bf16* vv = ws<__bf16>("ly_vv_h", (size_t)R * 12 * h);
      __bf16* oa = ws<__bf16>("ly_oa_h", (size_t)R * 12 * h);
      linear_h(Ly.sa_in[k], X, false, d, R, vv, true, 12 * h, EPI_NONE);
      AttnFlashArgs a = fa;
      a.v = vv;
      a.out = oa;
      prof_begin("attn_apply");
      launch_attn_flash(a, k == 0 ? 1 : 2, st_);
      prof_end();
      linear_h(Ly.sa_out[k], oa, true, 12 * h, R, X, false, d, EPI_RESADD);
      return;
    }
    float* vv = ws<float>("ly_vv", (size_t)R * 12 * h);
    float* oa = ws<float>("ly_oa", (size_t)R * 12 * h);
    linear(Ly.sa_in[k], X, d, R, vv, 12 * h, EPI_NONE);
    if (np) {
      AttnFlashArgs a = fa;
      a.v = vv;
      a.out = oa;
      prof_begin("attn_apply");
      launch_attn_flash(a, k == 0 ? 1 : 2, st_);
      prof_end();
      linear(Ly.sa_out[k], oa, 12 * h, R, X, d, EPI_RESADD);
      return;
    }
    AttnSAArgs sa{qkp, h, Ly.pos_tab, model_.pmax, d_off, B, maxL, stats, vv, oa, stats};
    prof_begin("attn_apply");
    launch_attn_sa(sa, k == 0, false, st_);
    prof_end();
    linear(Ly.sa_out[k], oa, 12 * h, R, X, d, EPI_RESADD);
  };
  auto conv = [&](int k) {
    if (Ly.cv_in[k].wh) {  // bf16 mode: in_proj output and out_proj input in bf16
      __bf16* dc = ws<__bf16>("ly_dc_h", (size_t)R * d);
      if (Ly.cv_in[k].glu) {  // the GLU in the in_proj epilogue (f32, then bf16), d columns
        __bf16* g = ws<__bf16>("ly_glu_h", (size_t)R * d);
        linear_h(Ly.cv_in[k], X, false, d, R, g, true, d, EPI_GLU);
        prof_begin("dwconv1d");
        launch_dwconv1d_post_glu_bf16(g, d_off, d_map, R, d, S.K, Ly.cv_dw_w[k], Ly.cv_dw_b[k], dc, st_);
        prof_end();
      } else {
        __bf16* g2 = ws<__bf16>("ly_g2_h", (size_t)R * 2 * d);
        linear_h(Ly.cv_in[k], X, false, d, R, g2, true, 2 * d, EPI_NONE);
        prof_begin("dwconv1d");
        launch_glu_dwconv1d_bf16(g2, d_off, d_map, R, d, S.K, Ly.cv_dw_w[k], Ly.cv_dw_b[k], dc, st_);
        prof_end();
      }
      linear_h(Ly.cv_out[k], dc, true, d, R, X, false, d, EPI_RESADD);
      return;
    }
    float* dc = ws<float>("ly_dc", (size_t)R * d);
    if (Ly.cv_in[k].glu) {  // split modes: the GLU in the in_proj epilogue, d columns out
      float* g = ws<float>("ly_glu", (size_t)R * d);
      linear(Ly.cv_in[k], X, d, R, g, d, EPI_GLU);
      prof_begin("dwconv1d");
      launch_dwconv1d_post_glu(g, d_off, d_map, R, d, S.K, Ly.cv_dw_w[k], Ly.cv_dw_b[k], dc, st_);
      prof_end();
    } else {
      float* g2 = ws<float>("ly_g2", (size_t)R * 2 * d);
      linear(Ly.cv_in[k], X, d, R, g2, 2 * d, EPI_NONE);
      prof_begin("dwconv1d");
      launch_glu_dwconv1d(g2, d_off, d_map, R, d, S.K, Ly.cv_dw_w[k], Ly.cv_dw_b[k], dc, st_);
      prof_end();
    }
    linear(Ly.cv_out[k], dc, d, R, X, d, EPI_RESADD);
  };
  // 1. feed_forward1
  ff(0);
  // 2. nonlin_attention (attention head 0 only)
  if (bf16) {
    // z = (A0 @ t1) * y with t1^T [hid][R8] bf16, z bf16; (s, x, y) = chunk(in_proj(src), 3)
    // in bf16: s, x read by the transpose kernel, y by the fused kernel's epilogue
    __bf16* h3 = ws<__bf16>("ly_h3_h", (size_t)R * 3 * hid);
    __bf16* t1t = ws<__bf16>("ly_t1t", (size_t)hid * R8);
    __bf16* z = ws<__bf16>("ly_z_h", (size_t)R * hid);
    linear_h(Ly.na_in, X, false, d, R, h3, true, 3 * hid, EPI_NONE);
    prof_begin("elementwise");
    launch_nonlin_prep_t(h3, true, d_off, d_o8, d_map, R, hid, R8, t1t, st_);
    prof_end();
    // z = (A0 @ t1) * y in the flash kernel (mode 3): head 0's weights never reach HBM
    AttnFlashArgs a = fa;
    a.t1t = t1t;
    a.o8 = d_o8;
    a.ldt = R8;
    a.hid = hid;
    a.y = h3 + 2 * hid;
    a.ldy = 3 * hid;
    a.z = z;
    prof_begin("attn_nonlin");
    launch_attn_flash(a, 3, st_);
    prof_end();
    linear_h(Ly.na_out, z, true, hid, R, X, false, d, EPI_RESADD);
  } else if (np) {
    // z = (A0 @ t1) * y on the split-bf16 GEMM: A0 [L][L8] f32 (split while staging),
    // t1^T as np bf16 pieces [np][hid][R8] (the weight layout), y f32 in the epilogue
    float* h3 = ws<float>("ly_h3", (size_t)R * 3 * hid);
    __bf16* t1t = ws<__bf16>("ly_t1t_x", (size_t)stored_pieces(np) * hid * R8);
    float* z = ws<float>("ly_z", (size_t)R * hid);
    linear(Ly.na_in, X, d, R, h3, 3 * hid, EPI_NONE);
    prof_begin("elementwise");
    launch_nonlin_prep_t(h3, false, d_off, d_o8, d_map, R, hid, R8, t1t, st_, np);
    prof_end();
    if (np == kPiecesF16) {
      // f16x3: z = (A0 @ t1) * y in the flash kernel (mode 3, fp16 pieces of P and t1)
      AttnFlashArgs a = fa;
      a.t1t = t1t;
      a.o8 = d_o8;
      a.ldt = R8;
      a.hid = hid;
      a.y = h3 + 2 * hid;
      a.ldy = 3 * hid;
      a.z = z;
      prof_begin("attn_nonlin");
      launch_attn_flash(a, 3, st_);
      prof_end();
    } else {
    GemmParams p{};
    p.A = A;
    p.B = nullptr;
    p.sbk = 1;
    p.sbn = R8;
    p.C = z;
    p.ldc = hid;
    p.N = hid;
    p.alpha = 1.f;
    p.aux = h3 + 2 * hid;
    p.ldaux = 3 * hid;
    p.slices = reinterpret_cast<const GemmSlice*>(d_slices_nl);
    p.num_slices = B;
    p.max_M = maxL;
    prof_begin("attn_nonlin");
    gemm_x3(p, t1t, (long)hid * R8, EPI_MULAUX, ALOAD_DENSE, st_, np);
    prof_end();
    }
    linear(Ly.na_out, z, hid, R, X, d, EPI_RESADD);
  } else {
    float* h3 = ws<float>("ly_h3", (size_t)R * 3 * hid);
    float* t1 = ws<float>("ly_t1", (size_t)R * hid);
    float* z = ws<float>("ly_z", (size_t)R * hid);
    linear(Ly.na_in, X, d, R, h3, 3 * hid, EPI_NONE);
    prof_begin("elementwise");
    launch_nonlin_prep(h3, t1, R, hid, st_);
    prof_end();
    GemmParams p{};
    p.A = A;
    p.B = t1;
    p.sbk = hid;
    p.sbn = 1;
    p.C = z;
    p.ldc = hid;
    p.N = hid;
    p.alpha = 1.f;
    p.aux = h3 + 2 * hid;
    p.ldaux = 3 * hid;
    p.slices = reinterpret_cast<const GemmSlice*>(d_slices_nl);
    p.num_slices = B;
    p.max_M = maxL;
    prof_begin("attn_nonlin");
    gemm_f32(p, EPI_MULAUX, ALOAD_DENSE, true, st_);
    prof_end();
    linear(Ly.na_out, z, hid, R, X, d, EPI_RESADD);
  }
  // 3. self_attn1, conv_module1, feed_forward2
  self_attn(0);
  conv(0);
  ff(1);
  // 4. bypass_mid (bf16 and split modes: folded into feed_forward2's epilogue)
  if (!bf16 && Ly.ff_out[1].wx == nullptr) {
    prof_begin("elementwise");
    launch_bypass(X, O, Ly.bypass_mid, R, d, st_);
    prof_end();
  }
  // 5. self_attn2, conv_module2, feed_forward3
  self_attn(1);
  conv(1);
  ff(2);
  // 6. BiasNorm + bypass (folding it into feed_forward3's fused epilogue -- the row's sums of
  // squares reduced across the block's waves, X read twice -- measured slower: ffn_fused
  // +1.26 ms, elementwise -0.78 ms per hour)
  prof_begin("elementwise");
  launch_bias_norm(X, R, d, Ly.norm_b, Ly.norm_ls, O, Ly.bypass, st_, last_layer ? nullptr : O);
  prof_end();
}

void Engine::run_encoder(const float* d_feats, const std::vector<int>& T, float* d_enc,
                         std::vector<int>& t_out) {
  const ModelConfig& cfg = model_.cfg;
  const int B = (int)T.size();
  std::vector<int> t1(B), l2(B), L(B), tout(B);
  for (int b = 0; b < B; ++b) {
    ZASR_REQUIRE(T[b] >= 9, "encoder needs >= 9 fbank frames per chunk");
    t1[b] = T[b] - 2;
    l2[b] = (T[b] - 3) / 2;
    L[b] = (T[b] - 7) / 2;
    tout[b] = (L[b] + 1) / 2;
  }
  t_out = tout;
  LevelMeta mfb = make_level(T), mc1 = make_level(t1), mc2 = make_level(l2), mL = make_level(L),
            mout = make_level(tout);
  const int ns = (int)model_.stacks.size();
  std::vector<LevelMeta> mst(ns);
  std::vector<std::vector<long>> aoff(ns);
  std::vector<std::vector<GemmSlice>> sl_nl(ns);
  std::vector<std::vector<int>> o8(ns);
  std::vector<int> R8(ns, 0);
  const bool bf16 = precision_ == 1 || precision_ == 2;
  // the flash attention path (bf16 and the split-bf16 modes): head-0 weights with L32 rows
  // ("L8" / "o8" / "R8" below: 32-padded),
  // NonlinAttention's B operand as t1^T columns
  const bool flash = bf16 || split_pieces() > 0;
  size_t attn_floats = 0;
  int maxL_all = 0;
  for (int i = 0; i < ns; ++i) {
    const DStack& s = model_.stacks[i];
    std::vector<int> len(B);
    for (int b = 0; b < B; ++b) len[b] = (L[b] + s.ds - 1) / s.ds;
    mst[i] = make_level(len);
    maxL_all = std::max(maxL_all, mst[i].maxlen);
    long acc = 0;
    const int hid = 3 * s.d / 4;
    int c8 = 0;
    for (int b = 0; b < B; ++b) {
      const int Lb = len[b], L4 = (Lb + 3) & ~3, L8 = (Lb + 31) & ~31;
      // weight row stride (flash: the GEMM's K padding, 32 for the LDS-DMA nonlin GEMM)
      const int Lp = flash ? L8 : L4;
      aoff[i].push_back(acc);
      o8[i].push_back(c8);
      GemmSlice g{};
      g.a_off = acc;  // head 0 block of this sequence
      g.b_off = flash ? (long)c8 : (long)mst[i].off[b] * hid;  // flash: column of t1^T
      g.c_off = (long)mst[i].off[b] * hid;
      g.aux_off = (long)mst[i].off[b] * 3 * hid;
      g.M = Lb;
      g.K = flash ? L8 : Lb;
      g.lda = Lp;
      sl_nl[i].push_back(g);
      acc += (long)Lb * Lp;  // only head 0 is materialised (nonlin_attention)
      c8 += L8;
    }
    o8[i].push_back(c8);
    R8[i] = c8;
    attn_floats = std::max(attn_floats, (size_t)acc);
  }
  ensure_pos_tables(maxL_all + 192);  // the bf16 attention stages rows up to L + 160
  // frontend conv slices
  std::vector<GemmSlice> sl_c2(B), sl_c3(B);
  for (int b = 0; b < B; ++b) {
    sl_c2[b] = GemmSlice{(long)mc1.off[b] * 640, 0, (long)mc2.off[b] * 39 * 32, 0, l2[b] * 39, 72, 0, 0};
    sl_c3[b] = GemmSlice{(long)mc2.off[b] * 39 * 32, 0, (long)mL.off[b] * 19 * 128, 0, L[b] * 19, 288, 0, 0};
  }
  // one metadata upload
  MetaPack mp;
  size_t o_fb = mp.add(mfb.off.data(), (B + 1) * 4), o_c1 = mp.add(mc1.off.data(), (B + 1) * 4),
         o_L = mp.add(mL.off.data(), (B + 1) * 4), o_out = mp.add(mout.off.data(), (B + 1) * 4);
  size_t o_c2s = mp.add(sl_c2.data(), B * sizeof(GemmSlice)),
         o_c3s = mp.add(sl_c3.data(), B * sizeof(GemmSlice));
  std::vector<size_t> o_st(ns), o_ao(ns), o_sn(ns), o_o8(ns);
  for (int i = 0; i < ns; ++i) {
    o_st[i] = mp.add(mst[i].off.data(), (B + 1) * 4);
    o_o8[i] = mp.add(o8[i].data(), (B + 1) * 4);
    o_ao[i] = mp.add(aoff[i].data(), B * sizeof(long));
    o_sn[i] = mp.add(sl_nl[i].data(), sl_nl[i].size() * sizeof(GemmSlice));
  }
  char* d_meta = ws<char>("enc_meta", mp.bytes.size());
  upload(d_meta, mp.bytes.data(), mp.bytes.size());
  auto I = [&](size_t o) { return reinterpret_cast<const int*>(d_meta + o); };
  // row -> sequence maps of every resolution used by per-row kernels
  int* c1_map = ws<int>("map_c1", mc1.total);
  int* L_map = ws<int>("map_L", mL.total);
  int* out_map = ws<int>("map_out", mout.total);
  launch_row2seq(I(o_c1), B, mc1.total, c1_map, st_);
  launch_row2seq(I(o_L), B, mL.total, L_map, st_);
  launch_row2seq(I(o_out), B, mout.total, out_map, st_);
  std::vector<int*> st_map(ns);
  for (int i = 0; i < ns; ++i) {
    st_map[i] = ws<int>("map_st" + std::to_string(i), mst[i].total);
    launch_row2seq(I(o_st[i]), B, mst[i].total, st_map[i], st_);
  }

  // ---------------- Conv2dSubsampling ----------------
  // bf16 mode: conv.0 and conv.4 outputs in bf16 (read back through the GEMM's bf16
  // implicit-im2col loaders)
  const bool fe16 = model_.conv4.wh != nullptr && model_.conv7.wh != nullptr;
  void* c1 = fe16 ? (void*)ws<__bf16>("fe_c1_h", (size_t)mc1.total * 640)
                  : (void*)ws<float>("fe_c1", (size_t)mc1.total * 640);
  prof_begin("frontend_conv");
  launch_conv1(d_feats, I(o_fb), I(o_c1), c1_map, mc1.total, model_.conv0_w, model_.conv0_b, c1,
               fe16, st_, split_pieces() == kPiecesF16);
  prof_end();
  void* c2 = fe16 ? (void*)ws<__bf16>("fe_c2_h", (size_t)mc2.total * 39 * 32)
                  : (void*)ws<float>("fe_c2", (size_t)mc2.total * 39 * 32);
  {
    GemmParams p{};
    p.A = reinterpret_cast<const float*>(c1);
    p.B = model_.conv4.w;
    p.sbk = 1;
    p.sbn = 72;
    p.C = reinterpret_cast<float*>(c2);
    p.ldc = 32;
    p.bias = model_.conv4.b;
    p.N = 32;
    p.alpha = 1.f;
    p.slices = reinterpret_cast<const GemmSlice*>(d_meta + o_c2s);
    p.num_slices = B;
    p.max_M = mc2.maxlen * 39;
    prof_begin("frontend_conv");
    if (fe16)
      gemm_bf16(p, model_.conv4.wh, EPI_SWOOSHR, ALOAD_CONV2, st_, true, true);
    else if (model_.conv4.wx)
      gemm_x3(p, model_.conv4.wx, 32L * 72, EPI_SWOOSHR, ALOAD_CONV2, st_, split_pieces());
    else if (model_.conv4.wh)
      gemm_bf16(p, model_.conv4.wh, EPI_SWOOSHR, ALOAD_CONV2, st_);
    else
      gemm_f32(p, EPI_SWOOSHR, ALOAD_CONV2, false, st_);
    prof_end();
  }
  const int d0 = cfg.dims[0];
  float* e0 = ws<float>("fe_e0", (size_t)mL.total * d0);
  {
    GemmParams p{};
    p.A = reinterpret_cast<const float*>(c2);
    p.B = model_.conv7.w;
    p.sbk = 1;
    p.sbn = 288;
    p.ldc = 128;
    p.bias = model_.conv7.b;
    p.N = 128;
    p.alpha = 1.f;
    p.slices = reinterpret_cast<const GemmSlice*>(d_meta + o_c3s);
    p.num_slices = B;
    p.max_M = mL.maxlen * 19;
    if (model_.pw1.wh) {
      // bf16 mode: conv.7 output, the ConvNeXt block and its output stay bf16
      __bf16* x3 = ws<__bf16>("fe_x3_h", (size_t)mL.total * 19 * 128);
      __bf16* y3 = ws<__bf16>("fe_y3_h", (size_t)mL.total * 19 * 128);
      __bf16* x4 = ws<__bf16>("fe_x4_h", (size_t)mL.total * 19 * 128);
      p.C = reinterpret_cast<float*>(x3);
      prof_begin("frontend_conv");
      gemm_bf16(p, model_.conv7.wh, EPI_SWOOSHR, ALOAD_CONV3, st_, fe16, true);
      prof_end();
      prof_begin("frontend_conv");
      launch_convnext_bf16(x3, I(o_L), L_map, mL.total, model_.dw_w, model_.dw_b, model_.pw1.wp,
                           model_.pw1.b, model_.pw2.wp, model_.pw2.b, y3, x4, st_);
      prof_end();
      linear_h(model_.out, x4, true, 2432, mL.total, e0, false, d0, EPI_NONE);
    } else {
      float* x3 = ws<float>("fe_x3", (size_t)mL.total * 19 * 128);
      p.C = x3;
      prof_begin("frontend_conv");
      if (model_.conv7.wx)
        gemm_x3(p, model_.conv7.wx, 128L * 288, EPI_SWOOSHR, ALOAD_CONV3, st_, split_pieces());
      else
        gemm_f32(p, EPI_SWOOSHR, ALOAD_CONV3, false, st_);
      prof_end();
      float* y3 = ws<float>("fe_y3", (size_t)mL.total * 19 * 128);
      prof_begin("frontend_conv");
      launch_dwconv2d_tiled(x3, I(o_L), L_map, mL.total, model_.dw_w, model_.dw_b, y3, st_);
      prof_end();
      if (model_.pw1.wr && model_.pw2.wr) {
        // f16x3: the ConvNeXt MLP as the fused f16x3 FFN (d = 128, pw1.N hidden): x3 += MLP(y3)
        prof_begin("frontend_conv");
        launch_ffn_fused_h3(x3, mL.total * 19, 128, model_.pw1.N, model_.pw1.wr, model_.pw1.b,
                            model_.pw2.wr, model_.pw2.b, st_, nullptr, nullptr, y3);
        prof_end();
      } else if (model_.pw1.wp && model_.pw2.wp && split_pieces() == kPiecesF16) {
        // f16x3: pw1 -> SwooshL -> pw2 + residual in one kernel, the hidden layer on chip
        prof_begin("frontend_conv");
        launch_convnext_mlp_h3(y3, x3, (long)mL.total * 19, model_.pw1.wp, model_.pw1.b,
                               model_.pw2.wp, model_.pw2.b, x3, st_);
        prof_end();
      } else {
        float* hcn = ws<float>("fe_h", (size_t)mL.total * 19 * 384);
        linear(model_.pw1, y3, 128, mL.total * 19, hcn, 384, EPI_SWOOSHL);
        linear(model_.pw2, hcn, 384, mL.total * 19, x3, 128, EPI_RESADD);
      }
      linear(model_.out, x3, 2432, mL.total, e0, d0, EPI_NONE);
    }
  }
  prof_begin("elementwise");
  launch_bias_norm(e0, mL.total, d0, model_.out_norm_b, model_.out_norm_ls, nullptr, nullptr, st_);
  prof_end();

  // ---------------- encoder stacks ----------------
  if (bf16)  // (the fused NonlinAttention never materialises head 0's weights)
    ws<__bf16>("ly_attn_h", 1);
  else
    ws<float>("ly_attn", split_pieces() == kPiecesF16 ? 1 : std::max<size_t>(attn_floats, 1));
  const int Dm = cfg.max_dim();
  float* full = ws<float>("st_full", (size_t)mL.total * Dm);
  // stack i's input (50 Hz, width d_i): stack 0 takes the embed output, every later one is
  // written by the previous seam's stack_glue
  float* orig = ws<float>("st_orig0", (size_t)mL.total * model_.stacks[0].d);
  prof_begin("elementwise");
  launch_copy_cols(e0, d0, 0, orig, model_.stacks[0].d, 0, std::min(d0, model_.stacks[0].d),
                   mL.total, true, model_.stacks[0].d, st_);
  prof_end();
  for (int i = 0; i < ns; ++i) {
    const DStack& s = model_.stacks[i];
    const int d = s.d;
    float* X;
    if (s.ds == 1) {
      X = orig;
    } else {
      X = ws<float>("st_x", (size_t)mst[i].total * d);
      prof_begin("elementwise");
      launch_downsample(orig, I(o_L), I(o_st[i]), st_map[i], mst[i].total, d, s.ds, s.ds_w, X, st_);
      prof_end();
    }
    for (size_t li = 0; li < s.layers.size(); ++li)
      layer_forward(s, s.layers[li], X, mst[i].total, I(o_st[i]), st_map[i], mst[i].len,
                    reinterpret_cast<const long*>(d_meta + o_ao[i]), d_meta + o_sn[i],
                    mst[i].maxlen, I(o_o8[i]), R8[i], li > 0, li + 1 == s.layers.size());
    // seam: upsample + bypass combine, written as stack i+1's input and into the full-dim
    // output's channel range [d_later_max, d) (the latest stack that has those channels)
    int later_max = 0;
    for (int j = i + 1; j < ns; ++j) later_max = std::max(later_max, model_.stacks[j].d);
    const int dn = i + 1 < ns ? model_.stacks[i + 1].d : 0;
    float* next = i + 1 < ns ? ws<float>("st_orig" + std::to_string((i + 1) % 2), (size_t)mL.total * dn)
                             : nullptr;
    prof_begin("elementwise");
    launch_stack_glue(X, orig, I(o_L), I(o_st[i]), L_map, mL.total, d, s.ds, s.comb, next, dn,
                      d > later_max ? full : nullptr, Dm, later_max, st_);
    prof_end();
    orig = next;
  }
  // ---------------- output downsample + encoder_proj ----------------
  float* fo = ws<float>("enc_ds", (size_t)mout.total * Dm);
  prof_begin("elementwise");
  launch_downsample(full, I(o_L), I(o_out), out_map, mout.total, Dm, 2, model_.out_ds_w, fo, st_);
  prof_end();
  linear(model_.enc_proj, fo, Dm, mout.total, d_enc, cfg.joiner_dim, EPI_NONE);
}

std::vector<TokenResult> Engine::run_search(const float* d_enc, const std::vector<int>& t_out,
                                            int beam) {
  SearchJob job;
  launch_search(d_enc, t_out, beam, 0, st_, true, job);
  return collect_search(job);
}

void Engine::launch_search(const float* d_enc, const std::vector<int>& t_out, int beam, int set,
                           hipStream_t stream, bool split_groups, SearchJob& job) {
  const ModelConfig& cfg = model_.cfg;
  const int S_all = (int)t_out.size();
  job = SearchJob{};
  job.S_all = S_all;
  job.t_out = t_out;
  job.set = set;
  job.stream = stream;
  hipStream_t caller_st = st_;
  const std::string caller_tag = ws_tag_;
  st_ = stream;
  ws_tag_ = set ? "q" + std::to_string(set) + "/" : "";  // set 0: the single-search names
  pin_reset(kMaxEnc + 1 + set);
  struct Restore {
    Engine* e;
    hipStream_t st;
    std::string tag;
    ~Restore() {
      e->st_ = st;
      e->ws_tag_ = tag;
    }
  } restore{this, caller_st, caller_tag};
  // streams with T' >= 1, sorted by T' descending so active streams form a prefix
  std::vector<int> order;
  std::vector<int> enc_off_all(S_all + 1, 0);
  for (int s = 0; s < S_all; ++s) enc_off_all[s + 1] = enc_off_all[s] + t_out[s];
  for (int s = 0; s < S_all; ++s)
    if (t_out[s] > 0) order.push_back(s);
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return t_out[a] > t_out[b]; });
  const int S = (int)order.size();
  job.S = S;
  job.check_finite = precision_ == 5;
  if (S == 0) return;
  const int H = beam;
  const int Tmax = t_out[order[0]];
  const int V = cfg.V, D = cfg.joiner_dim;
  std::vector<int> eo(S), el(S);
  for (int i = 0; i < S; ++i) {
    eo[i] = enc_off_all[order[i]];
    el[i] = t_out[order[i]];
  }
  int* d_eo = ws<int>("se_eo", S);
  int* d_el = ws<int>("se_el", S);
  upload(d_eo, eo.data(), S * sizeof(int));
  upload(d_el, el.data(), S * sizeof(int));
  const size_t slots = (size_t)S * H;
  SearchState st{};
  st.lp = ws<double>("se_lp", slots);
  st.lpf = ws<int>("se_lpf", slots);
  st.hash = ws<unsigned long long>("se_hash", slots);
  st.len = ws<int>("se_len", slots);
  st.y1 = ws<int>("se_y1", slots);
  st.y2 = ws<int>("se_y2", slots);
  st.hw = ws<int>("se_hw", slots);
  st.node = ws<int>("se_node", slots);
  st.nh = ws<int>("se_nh", S);
  st.node_cap = H * Tmax + 1;
  const size_t ncap = (size_t)S * st.node_cap;
  st.node_tok = ws<int>("se_ntok", ncap);
  st.node_frame = ws<int>("se_nfr", ncap);
  st.node_parent = ws<int>("se_npar", ncap);
  st.node_lp = ws<double>("se_nlp", ncap);
  st.node_stats = ws<float4>("se_nst", ncap);
  st.node_count = ws<int>("se_ncnt", S);
  float* logits = ws<float>("se_logits", slots * V);
  // split-bf16 modes: J written once as `np` packed bf16 pieces (store_j4), the joiner on the
  // packed W pieces; bf16: one packed bf16 image
  const int jnp = split_pieces();
  const bool bf16 = model_.joiner.wh != nullptr;
  // bf16 with the decoder-context table: J in fragment order for the packed joiner (every
  // J writer goes through store_j4); without the table decjoin writes row-major J
  const bool packed = (bf16 || jnp > 0) && model_.joiner_packed && model_.dec_table;
  const int jpc = packed && jnp > 0 ? stored_pieces(jnp) : 1;  // packed images of J
  const bool j16 = bf16 || packed;              // J buffer in bf16 elements
  const size_t jrows = (size_t)joiner_packed_rows((long)slots);
  void* J = j16 ? (void*)ws<__bf16>("se_joinin_h", jrows * D * jpc) : (void*)ws<float>("se_joinin", slots * D);
  ZASR_HIP_CHECK(hipMemsetAsync(J, 0, (j16 ? jrows * 2 * jpc : slots * 4) * D, st_));
  DecTable dt{model_.dec_table, V, d_enc, d_eo, d_el, J, D, bf16 ? 1 : 0};
  dt.j_packed = packed ? 1 : 0;
  dt.j_pieces = packed ? jnp : 0;
  dt.j_plane = (long)jrows * D;
  auto packed_args = [&](const void* Jp, long jplane, float* out, int rows) {
    JoinerPackedArgs ja{Jp, model_.joiner_packed, model_.joiner.b, out, rows, V, D};
    if (jnp > 0) {
      ja.pieces = jnp;
      ja.j_plane = jplane;
      ja.w_plane = model_.joiner_plane;
    }
    return ja;
  };
  DecoderW dw{model_.dec_tap0, model_.dec_tap1, model_.dec_proj.b, D};
  // greedy with the decoder-context table: speculative windows (kernels.h, greedy_spec)
  const char* spec_env = getenv("ZASR_GREEDY_WINDOW");
  const int F = spec_env ? atoi(spec_env) : 4;
  if (H == 1 && model_.dec_table && (F == 4 || F == 8)) {
    const size_t jrs = (size_t)joiner_packed_rows((long)S * F);
    void* Js = j16 ? (void*)ws<__bf16>("gs_joinin_h", jrs * D * jpc)
                   : (void*)ws<float>("gs_joinin", (size_t)S * F * D);
    // ZASR_GREEDY_FUSED=1: one launch per super-step (joiner_greedy_kernel, packed bf16 / f16x3
    // joiner, F = 4), bit-identical to the two launches but measured slower: per super-step
    // 22.8 vs 21.0 us of kernel time, and its 8-wave blocks at 219 VGPRs crowd the next batch's
    // encoder out (pipelined bf16 hour 104.7k vs 120.8k xRT, profiles/r06/fused_greedy/,
    // DESIGN.md §11) -- the write-through hand-off and the last-arriver's one wave per stream
    // cost what the launch boundary did.  Default: joiner + greedy_spec
    static const bool fused_env = getenv("ZASR_GREEDY_FUSED") && getenv("ZASR_GREEDY_FUSED")[0] == '1';
    const bool fused = fused_env && packed && F == 4 && (jnp == 0 || jnp == kPiecesF16) &&
                       (D == 256 || D == 512) && V % 4 == 0 && V <= 2048;
    const int ldo = fused ? joiner_greedy_ldo(V) : V;
    float* lg = ws<float>("gs_logits", (size_t)S * F * ldo);
    int* d_t = ws<int>("gs_t", S);
    int* d_active = ws<int>("gs_active", 2);
    int* d_cnt = fused ? ws<int>("gs_cnt", (size_t)cdiv(S, 8)) : nullptr;
    DecTable ds{model_.dec_table, V, d_enc, d_eo, d_el, Js, D, bf16 ? 1 : 0};
    ds.j_packed = packed ? 1 : 0;
    ds.j_pieces = packed ? jnp : 0;
    ds.j_plane = (long)jrs * D;
    prof_begin("search");
    launch_search_init(st, S, 1, st_);
    launch_greedy_spec_init(ds, S, F, d_t, d_active, st_);
    if (fused) ZASR_HIP_CHECK(hipMemsetAsync(d_cnt, 0, (size_t)cdiv(S, 8) * sizeof(int), st_));
    prof_end();
    // every super-step advances each live stream by >= 1 frame: Tmax steps at most; the
    // host checks the live-stream count every kSync steps (one small D2H copy)
    constexpr int kSync = 16;
    int k = 0;
    hipEvent_t live_ev[2];
    for (auto& e : live_ev) ZASR_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    int slot = 0;
    bool have_prev = false;
    while (k < Tmax) {
      for (int b = 0; b < kSync && k < Tmax; ++b, ++k) {
        if (fused) {
          GreedyFusedArgs ga{};
          ga.j = packed_args(Js, ds.j_plane, lg, S * F);
          ga.ldo = ldo;
          ga.st = st;
          ga.t_cur = d_t;
          ga.enc_len = d_el;
          ga.hw = hw_;
          ga.dt = ds;
          ga.active = d_active;
          ga.parity = k & 1;
          ga.cnt = d_cnt;
          ga.S = S;
          prof_begin("joiner_search");
          launch_joiner_greedy(ga, st_);
          prof_end();
          continue;
        }
        prof_begin("joiner");
        if (packed) {
          JoinerPackedArgs ja = packed_args(Js, ds.j_plane, lg, S * F);
          ja.live_t = d_t;
          ja.live_len = d_el;
          ja.live_f = F;
          launch_joiner_packed(ja, st_);
        } else if (bf16) {
          JoinerBf16Args ja{reinterpret_cast<const __bf16*>(Js),
                            reinterpret_cast<const __bf16*>(model_.joiner.wh), model_.joiner.b, lg,
                            S * F, V, D, d_t, d_el, F};
          launch_joiner_bf16(ja, st_);
        } else {
          JoinerArgs ja{reinterpret_cast<const float*>(Js), model_.joiner.w, model_.joiner.b, lg,
                        S * F, V, D, d_t, d_el, F};
          ja.Wx = reinterpret_cast<const __bf16*>(model_.joiner.wx);
          ja.pieces = split_pieces();
          launch_joiner(ja, st_);
        }
        prof_end();
        prof_begin("search");
        launch_greedy_spec(st, lg, V, S, F, d_t, d_el, hw_, ds, d_active, k & 1, st_);
        prof_end();
      }
      // the live count after this batch lands in pinned slot `slot`; the host then waits only
      // for the PREVIOUS batch's count, so the GPU always has the next kSync steps queued (a
      // batch enqueued after the last stream finished exits in every kernel's first lines)
      ZASR_HIP_CHECK(hipMemcpyAsync(h_pinned_ + slot, d_active + ((k - 1) & 1), sizeof(int),
                                    hipMemcpyDeviceToHost, st_));
      ZASR_HIP_CHECK(hipEventRecord(live_ev[slot], st_));
      if (have_prev) {
        ZASR_HIP_CHECK(hipEventSynchronize(live_ev[slot ^ 1]));
        if (h_pinned_[slot ^ 1] == 0) break;
      }
      have_prev = true;
      slot ^= 1;
    }
    for (auto e : live_ev) (void)hipEventDestroy(e);
  } else {
  // beam search: the streams are split into G groups whose frame chains run concurrently on
  // the two search streams (each group's chain is latency-bound: joiner -> search step per
  // frame; two chains interleave their launch and scheduling waits).  Group g holds the
  // streams order[g], order[g + G], ... (each group sorted by T' descending, active streams
  // a prefix), laid out contiguously; the search final runs over all of them.
  const int G = split_groups ? std::min(2, S) : 1;
  if (G > 1) {
    std::vector<int> reord;
    for (int g = 0; g < G; ++g)
      for (int i = g; i < S; i += G) reord.push_back(order[i]);
    order = reord;
    for (int i = 0; i < S; ++i) {
      eo[i] = enc_off_all[order[i]];
      el[i] = t_out[order[i]];
    }
    upload(d_eo, eo.data(), S * sizeof(int));
    upload(d_el, el.data(), S * sizeof(int));
  }
  struct Group {
    int s0, n;
    SearchState st;
    DecTable dt;
    void* J;
    float* logits;
    hipStream_t stream;
    int active;
  };
  std::vector<Group> grp(G);
  for (int g = 0, s0 = 0; g < G; ++g) {
    Group& q = grp[g];
    q.s0 = s0;
    q.n = (S - g + G - 1) / G;
    s0 += q.n;
    q.st = st;
    const size_t so = (size_t)q.s0 * H, no = (size_t)q.s0 * st.node_cap;
    q.st.lp += so; q.st.lpf += so; q.st.hash += so; q.st.len += so; q.st.y1 += so; q.st.y2 += so;
    q.st.hw += so; q.st.node += so; q.st.nh += q.s0;
    q.st.node_tok += no; q.st.node_frame += no; q.st.node_parent += no; q.st.node_lp += no;
    q.st.node_stats += no; q.st.node_count += q.s0;
    q.stream = g == 0 ? st_ : stream3_;
    if (g == 0) {
      q.J = J;
      q.logits = logits;
    } else {
      const size_t jr = (size_t)joiner_packed_rows((long)q.n * H);
      q.J = j16 ? (void*)ws<__bf16>("se_joinin_h1", jr * D * jpc) : (void*)ws<float>("se_joinin1", (size_t)q.n * H * D);
      q.logits = ws<float>("se_logits1", (size_t)q.n * H * V);
    }
    q.dt = dt;
    q.dt.enc_off = d_eo + q.s0;
    q.dt.enc_len = d_el + q.s0;
    q.dt.J = q.J;
    if (g > 0) q.dt.j_plane = (long)joiner_packed_rows((long)q.n * H) * D;
    q.active = q.n;
  }
  if (G > 1) {  // group 1 starts after the uploads / memsets / encoder-output wait on st_
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 3], st_));
    ZASR_HIP_CHECK(hipStreamWaitEvent(stream3_, part_ev_[kMaxEnc + 3], 0));
    const size_t jr = (size_t)joiner_packed_rows((long)grp[1].n * H);
    ZASR_HIP_CHECK(hipMemsetAsync(grp[1].J, 0, (j16 ? jr * 2 * jpc : (size_t)grp[1].n * H * 4) * D, stream3_));
  }
  hipStream_t home = st_;
  for (Group& q : grp) {
    st_ = q.stream;
    prof_begin("search");
    launch_search_init(q.st, q.n, H, st_);
    if (model_.dec_table) launch_table_init(q.dt, q.n, H, st_);
    prof_end();
  }
  // per frame and group: [decoder + J when there is no table] -> joiner -> search step (which
  // writes the next frame's J from the table)
  for (int t = 0; t < Tmax; ++t) {
    for (Group& q : grp) {
      const int* qel = el.data() + q.s0;
      while (q.active > 0 && qel[q.active - 1] <= t) --q.active;
      if (q.active == 0) continue;
      st_ = q.stream;
      const int rows = q.active * H;
      if (!model_.dec_table) {
        DecJoinArgs da{dw, model_.dec_proj.w, q.st.y1, q.st.y2, d_enc, d_eo + q.s0, q.J, rows, H, t, bf16 ? 1 : 0};
        prof_begin("decoder");
        launch_decjoin(da, st_);
        prof_end();
      }
      prof_begin("joiner");
      if (packed) {
        JoinerPackedArgs ja = packed_args(q.J, q.dt.j_plane, q.logits, rows);
        launch_joiner_packed(ja, st_);
      } else if (bf16) {
        JoinerBf16Args ja{reinterpret_cast<const __bf16*>(q.J), reinterpret_cast<const __bf16*>(model_.joiner.wh),
                          model_.joiner.b, q.logits, rows, V, D};
        launch_joiner_bf16(ja, st_);
      } else {
        JoinerArgs ja{reinterpret_cast<const float*>(q.J), model_.joiner.w, model_.joiner.b, q.logits, rows, V, D};
        ja.Wx = reinterpret_cast<const __bf16*>(model_.joiner.wx);
        ja.pieces = split_pieces();
        launch_joiner(ja, st_);
      }
      prof_end();
      prof_begin("search");
      launch_search_step(q.st, q.logits, V, q.active, H, beam, t, d_el + q.s0, hw_,
                         model_.dec_table ? &q.dt : nullptr, st_);
      prof_end();
    }
  }
  st_ = home;
  if (G > 1) {  // the final pick on st_ reads every group's nodes
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 3], stream3_));
    ZASR_HIP_CHECK(hipStreamWaitEvent(st_, part_ev_[kMaxEnc + 3], 0));
  }
  }
  const int cap = Tmax;
  job.cap = cap;
  job.Tmax = Tmax;
  job.order = order;
  int* o_tok = ws<int>("so_tok", (size_t)S * cap);
  int* o_fr = ws<int>("so_fr", (size_t)S * cap);
  double* o_lp = ws<double>("so_lp", (size_t)S * cap);
  float4* o_st = ws<float4>("so_st", (size_t)S * cap);
  int* o_cnt = ws<int>("so_cnt", S);
  prof_begin("search");
  launch_search_final(st, S, H, hw_, cap, o_tok, o_fr, o_lp, o_st, o_cnt, st_);
  prof_end();
  // results into this set's pinned buffers (a copy into pageable memory would block the host
  // until the search is done): [cnt S][tok S cap][fr S cap][lp S cap][stats S cap]
  const size_t n = (size_t)S * cap;
  const size_t bytes = 16 * n + 8 * n + 4 * n + 4 * n + 4 * (size_t)S + 64;
  ResPin& rp = res_pin_[set];
  if (rp.cap < bytes) {  // the set's previous job was collected: its buffer is free
    if (rp.p) ZASR_HIP_CHECK(hipHostFree(rp.p));
    rp.cap = bytes + bytes / 4;
    ZASR_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&rp.p), rp.cap, hipHostMallocDefault));
  }
  char* h = rp.p;
  ZASR_HIP_CHECK(hipMemcpyAsync(h, o_st, n * 16, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(h + 16 * n, o_lp, n * 8, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(h + 24 * n, o_tok, n * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(h + 28 * n, o_fr, n * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(h + 32 * n, o_cnt, (size_t)S * 4, hipMemcpyDeviceToHost, st_));
  if (job.check_finite) {
    // f16x3: the encoder output this search read must be finite (fp16 range guard)
    int* d_bad = ws<int>("so_nonfinite", 1);
    launch_nonfinite_check(d_enc, (long)enc_off_all[S_all] * D, d_bad, st_);
    ZASR_HIP_CHECK(hipMemcpyAsync(h + 32 * n + 4 * (size_t)S, d_bad, 4, hipMemcpyDeviceToHost, st_));
  }
  ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 4 + set], st_));
}

std::vector<TokenResult> Engine::collect_search(SearchJob& job) {
  std::vector<TokenResult> res(job.S_all);
  for (int s = 0; s < job.S_all; ++s) res[s].t_out = job.t_out[s];
  if (job.S == 0) return res;
  ZASR_HIP_CHECK(hipEventSynchronize(part_ev_[kMaxEnc + 4 + job.set]));
  const int S = job.S, cap = job.cap;
  const size_t n = (size_t)S * cap;
  const char* h = res_pin_[job.set].p;
  const float* h_st = reinterpret_cast<const float*>(h);
  const double* h_lp = reinterpret_cast<const double*>(h + 16 * n);
  const int* h_tok = reinterpret_cast<const int*>(h + 24 * n);
  const int* h_fr = reinterpret_cast<const int*>(h + 28 * n);
  const int* h_cnt = reinterpret_cast<const int*>(h + 32 * n);
  if (job.check_finite && h_cnt[S] != 0) {
    // drain every engine stream (later batches' encoders, the other search job) before the
    // error leaves the pipeline: the next call reuses the workspaces and pinned arenas
    ZASR_HIP_CHECK(hipDeviceSynchronize());
    throw std::runtime_error("precision f16x3: non-finite encoder output (an activation exceeded "
                             "the fp16 range of the split operands); decode with bf16x6 or fp32");
  }
  for (int i = 0; i < S; ++i) {
    TokenResult& r = res[job.order[i]];
    const int c = h_cnt[i];
    const size_t o = (size_t)i * cap;
    r.tok.assign(h_tok + o, h_tok + o + c);
    r.frame.assign(h_fr + o, h_fr + o + c);
    r.lp.assign(h_lp + o, h_lp + o + c);
    r.stats.assign(h_st + 4 * o, h_st + 4 * (o + c));
  }
  return res;
}

// ------------------------------------------------------------------------------------
// public entry points
// ------------------------------------------------------------------------------------
void Engine::encode_stage(const float* d_wav, const std::vector<long>& wav_off,
                          const std::vector<long>& n, int out_slot, int ws_slot,
                          hipStream_t stream, Pending& pd) {
  st_ = stream;
  pin_reset(out_slot);
  ws_tag_ = ws_slot ? "w" + std::to_string(ws_slot) + "/" : "";
  const int B = (int)n.size();
  pd = Pending{};
  pd.B = B;
  pd.ready = part_ev_[out_slot];
  std::vector<int> frames;
  long total_frames = 0;
  for (int b = 0; b < B; ++b) total_frames += n[b] > 0 ? (n[b] + 80) / 160 : 0;
  float* feats = ws<float>("feats", (size_t)std::max<long>(total_frames, 1) * 80);
  std::vector<long> off_dev(wav_off);
  if (host_wav_) {
    // this batch's span of the host signal -> the output slot's device buffer, on the copy
    // stream; the slot's previous batch has been searched, so its fbank is done with the buffer
    long lo = -1, hi = 0;
    for (int b = 0; b < B; ++b)
      if (n[b] > 0) {
        lo = lo < 0 ? wav_off[b] : std::min(lo, wav_off[b]);
        hi = std::max(hi, wav_off[b] + n[b]);
      }
    if (lo >= 0) {
      float* buf = ws<float>("wav_in" + std::to_string(out_slot), (size_t)(hi - lo));
      if (!copy_st_) ZASR_HIP_CHECK(hipStreamCreateWithFlags(&copy_st_, hipStreamNonBlocking));
      if (!upload_ev_[out_slot])
        ZASR_HIP_CHECK(hipEventCreateWithFlags(&upload_ev_[out_slot], hipEventDisableTiming));
      ZASR_HIP_CHECK(hipMemcpyAsync(buf, host_wav_ + lo, (size_t)(hi - lo) * sizeof(float),
                                    hipMemcpyHostToDevice, copy_st_));
      ZASR_HIP_CHECK(hipEventRecord(upload_ev_[out_slot], copy_st_));
      ZASR_HIP_CHECK(hipStreamWaitEvent(st_, upload_ev_[out_slot], 0));
      for (int b = 0; b < B; ++b) off_dev[b] = n[b] > 0 ? wav_off[b] - lo : 0;
      d_wav = buf;
    }
  }
  run_fbank(d_wav, off_dev, n, feats, frames);
  // chunks too short for the encoder produce empty results (T' = 0)
  std::vector<int> T;
  std::vector<long> foff(B + 1, 0);
  for (int b = 0; b < B; ++b) foff[b + 1] = foff[b] + frames[b];
  for (int b = 0; b < B; ++b)
    if (frames[b] >= 9) {
      pd.valid.push_back(b);
      T.push_back(frames[b]);
    }
  if (pd.valid.empty()) {
    ws_tag_.clear();
    return;
  }
  const float* fptr = feats;
  if ((int)pd.valid.size() != B) {  // compact valid chunks' features
    float* cf = ws<float>("feats_compact", (size_t)total_frames * 80);
    long pos = 0;
    for (int b : pd.valid) {
      ZASR_HIP_CHECK(hipMemcpyAsync(cf + pos * 80, feats + foff[b] * 80, (size_t)frames[b] * 80 * 4,
                                    hipMemcpyDeviceToDevice, st_));
      pos += frames[b];
    }
    fptr = cf;
  }
  long tot_out = 0;
  for (int t : T) tot_out += ((t - 7) / 2 + 1) / 2;
  // the encoder output is the only buffer the search reads: one per pipeline slot
  pd.enc = ws<float>("enc_out" + std::to_string(out_slot),
                     (size_t)std::max<long>(tot_out, 1) * model_.cfg.joiner_dim);
  run_encoder(fptr, T, pd.enc, pd.t_out);
  ZASR_HIP_CHECK(hipEventRecord(pd.ready, st_));
  ws_tag_.clear();
}

std::vector<TokenResult> Engine::search_stage(Pending& pd, int beam) {
  std::vector<TokenResult> out(pd.B);
  if (pd.valid.empty()) return out;
  hipStream_t main_st = st_;
  st_ = stream2_;
  ZASR_HIP_CHECK(hipStreamWaitEvent(stream2_, pd.ready, 0));
  std::vector<TokenResult> r = run_search(pd.enc, pd.t_out, beam);
  for (size_t i = 0; i < pd.valid.size(); ++i) out[pd.valid[i]] = std::move(r[i]);
  // the call's stream sees the search complete (its results are already on the host)
  ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 1], stream2_));
  ZASR_HIP_CHECK(hipStreamWaitEvent(main_st, part_ev_[kMaxEnc + 1], 0));
  st_ = main_st;
  return out;
}

std::vector<TokenResult> Engine::decode_device(const float* d_wav, const std::vector<long>& wav_off,
                                               const std::vector<long>& n, int beam,
                                               hipStream_t st) {
  return decode_device_batches(d_wav, wav_off, n, {(int)n.size()}, beam, st);
}

std::vector<TokenResult> Engine::decode_host_batches(const float* h_wav,
                                                     const std::vector<long>& wav_off,
                                                     const std::vector<long>& n,
                                                     const std::vector<int>& batch_sizes,
                                                     int beam, hipStream_t st) {
  struct Reset {
    const float** p;
    ~Reset() { *p = nullptr; }
  } reset{&host_wav_};
  host_wav_ = h_wav;
  return decode_device_batches(nullptr, wav_off, n, batch_sizes, beam, st);
}

std::vector<TokenResult> Engine::decode_device_batches(const float* d_wav,
                                                       const std::vector<long>& wav_off,
                                                       const std::vector<long>& n,
                                                       const std::vector<int>& batch_sizes,
                                                       int beam, hipStream_t st) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  long total = 0;
  for (int c : batch_sizes) {
    ZASR_REQUIRE(c >= 0, "negative batch size");
    total += c;
  }
  ZASR_REQUIRE(total == (long)n.size() && wav_off.size() == n.size(),
               "batch sizes must sum to the chunk count");
  hipStream_t main_st = st ? st : stream_;
  st_ = main_st;
  std::vector<TokenResult> out;
  out.reserve(n.size());
  // E encoder streams; L (= E + 1 by default, below) batches' encoders are enqueued ahead of
  // the search in flight.
  // Batch k: encoder output / event / pinned arena slot k % (L + 1), stream + workspace set
  // k % E.  When batch k + L is enqueued, the previous user of its output slot (batch k - 1)
  // has been searched (the search returns on the host), and its stream's previous batch
  // (k + L - E) is ordered before it on the same stream.
  // Greedy: the encoder is the critical path, a second encoder stream fills its kernel tails
  // (98.4k vs 95.3k xRT).  Beam search: the search is the critical path and a second encoder
  // stream only adds contention for it (69.9k vs 68.3k xRT at beam 8 + 20 hotwords).
  static const int env_e = getenv("ZASR_ENC_STREAMS") ? atoi(getenv("ZASR_ENC_STREAMS")) : 0;
  const int nb = (int)batch_sizes.size();
  // Beam search: several batches' searches in flight (ZASR_SEARCH_JOBS, default 2).  Each
  // batch's frame chain is latency-bound (joiner -> search step per frame, a few hundred
  // blocks), so further chains on the other search streams run beside it at nearly the same
  // per-frame latency.
  static const int env_jobs = getenv("ZASR_SEARCH_JOBS") ? atoi(getenv("ZASR_SEARCH_JOBS")) : 2;
  if (beam > 1 && env_jobs >= 2 && nb >= 2 && search_cus_ == 0)
    return decode_batches_two_searches(d_wav, wav_off, n, batch_sizes, beam, main_st);
  const int want_e = env_e ? env_e : (beam > 1 ? 1 : 2);
  const int E = std::max(1, std::min({want_e, (int)kMaxEnc, nb - 1}));
  // a second encoder stream: the persistent kernels leave 1/8 of the CUs to it (common.h)
  const PersistShare share(E > 1);
  // L: batches whose encoders are queued ahead of the search in flight, one more than the
  // encoder streams (at most kMaxEnc: L + 1 output slots): 111.8-113.1k -> 113.5-114.3k xRT
  // on one box (profiles/r03/enc_ahead/)
  const int L = std::max(E, std::min({E + 1, (int)kMaxEnc, nb}));
  // encoder stream 0 is the caller's stream, or (CU-partitioned) the engine's masked stream
  hipStream_t enc_st[kMaxEnc] = {search_cus_ > 0 ? stream_ : main_st};
  for (int e = 1; e < kMaxEnc; ++e) enc_st[e] = enc_extra_[e - 1];
  if (E > 1 || enc_st[0] != main_st) {  // the encoder streams start after the caller's prior work
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 2], main_st));
    for (int e = 0; e < E; ++e)
      if (enc_st[e] != main_st) ZASR_HIP_CHECK(hipStreamWaitEvent(enc_st[e], part_ev_[kMaxEnc + 2], 0));
  }
  std::vector<long> first(nb + 1, 0);
  for (int k = 0; k < nb; ++k) first[k + 1] = first[k] + batch_sizes[k];
  Pending pd[kMaxEnc + 1];
  auto enqueue = [&](int k) {
    std::vector<long> o(wav_off.begin() + first[k], wav_off.begin() + first[k + 1]);
    std::vector<long> l(n.begin() + first[k], n.begin() + first[k + 1]);
    encode_stage(d_wav, o, l, k % (L + 1), k % E, enc_st[k % E], pd[k % (L + 1)]);
    st_ = main_st;
  };
  for (int k = 0; k < std::min(L, nb); ++k) enqueue(k);
  for (int k = 0; k < nb; ++k) {
    if (k + L < nb) enqueue(k + L);
    std::vector<TokenResult> r = search_stage(pd[k % (L + 1)], beam);
    for (auto& x : r) out.push_back(std::move(x));
  }
  order_after_encoders(enc_st, E, main_st);
  st_ = stream_;
  return out;
}

void Engine::order_after_encoders(const hipStream_t* enc_st, int E, hipStream_t main_st) {
  // the caller's stream must not run ahead of an encoder stream that read its audio: a batch
  // without valid chunks is never searched, so nothing else orders its fbank / encoder work
  // (on a CU-masked stream_ or a second encoder stream) before the caller reuses the buffer
  for (int e = 0; e < E; ++e) {
    if (enc_st[e] == main_st) continue;
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 2], enc_st[e]));
    ZASR_HIP_CHECK(hipStreamWaitEvent(main_st, part_ev_[kMaxEnc + 2], 0));
  }
}

std::vector<TokenResult> Engine::decode_batches_two_searches(const float* d_wav,
                                                             const std::vector<long>& wav_off,
                                                             const std::vector<long>& n,
                                                             const std::vector<int>& batch_sizes,
                                                             int beam, hipStream_t main_st) {
  // J searches in flight (ZASR_SEARCH_JOBS, 2 or 3), L encoders enqueued ahead on E encoder
  // streams (ZASR_ENC_STREAMS, 1 or 2; default 1), J + L encoder output slots.  Batch k:
  // output slot / pinned arena k % (J + L), encoder stream and workspace set k % E, search job
  // set k % J on its own high-priority stream.  Per iteration k: start batch k's search,
  // collect batch k - J + 1's, enqueue batch k + L's encoder -- its slot was last used by
  // batch k - J (collected in iteration k - 1), its stream's previous batch k + L - E is
  // ordered before it on that stream, and job set k % J was last used by batch k - J.
  static const int env_jobs = getenv("ZASR_SEARCH_JOBS") ? atoi(getenv("ZASR_SEARCH_JOBS")) : 2;
  static const int env_e = getenv("ZASR_ENC_STREAMS") ? atoi(getenv("ZASR_ENC_STREAMS")) : 1;
  const int nb = (int)batch_sizes.size();
  const int J = std::max(2, std::min(env_jobs, (int)kMaxJobs));
  const int L = std::max(1, kMaxEnc + 1 - J);
  const int E = std::max(1, std::min(env_e, 2));
  // J searches beside the encoder: the persistent kernels leave 1/8 of the CUs to them
  // (config 3 in f16x3 58.5k -> 59.2k xRT, the drop-in phase within noise: 36.8k / 36.7k,
  // three interleaved pairs each, profiles/r06/persist_ab/beam_share.txt)
  const PersistShare share(true);
  const int NS = J + L;
  ZASR_REQUIRE(NS <= kMaxEnc + 1, "pipeline slots");
  hipStream_t enc_st[2] = {main_st, enc_extra_[0]};
  if (E > 1) {  // the second encoder stream starts after the caller's prior work
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 2], main_st));
    ZASR_HIP_CHECK(hipStreamWaitEvent(enc_st[1], part_ev_[kMaxEnc + 2], 0));
  }
  std::vector<long> first(nb + 1, 0);
  for (int k = 0; k < nb; ++k) first[k + 1] = first[k] + batch_sizes[k];
  Pending pd[kMaxEnc + 1];
  auto enqueue = [&](int k) {
    std::vector<long> o(wav_off.begin() + first[k], wav_off.begin() + first[k + 1]);
    std::vector<long> l(n.begin() + first[k], n.begin() + first[k + 1]);
    encode_stage(d_wav, o, l, k % NS, k % E, enc_st[k % E], pd[k % NS]);
    st_ = main_st;
  };
  struct Job {
    int B = 0;
    std::vector<int> valid;
    SearchJob sj;
    bool launched = false;
  } jobs[kMaxJobs];
  if (J > 2 && stream4_ == nullptr) {
    int least = 0, greatest = 0;
    ZASR_HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    ZASR_HIP_CHECK(hipStreamCreateWithPriority(&stream4_, hipStreamNonBlocking, greatest));
  }
  const hipStream_t sst[kMaxJobs] = {stream2_, stream3_, stream4_};
  auto start = [&](int k) {
    Pending& p = pd[k % NS];
    Job& j = jobs[k % J];
    j.B = p.B;
    j.valid = p.valid;
    j.launched = !p.valid.empty();
    if (!j.launched) return;
    ZASR_HIP_CHECK(hipStreamWaitEvent(sst[k % J], p.ready, 0));
    launch_search(p.enc, p.t_out, beam, k % J, sst[k % J], false, j.sj);
  };
  std::vector<TokenResult> out;
  out.reserve(n.size());
  auto finish = [&](int k) {
    Job& j = jobs[k % J];
    std::vector<TokenResult> o(j.B);
    if (j.launched) {
      std::vector<TokenResult> r = collect_search(j.sj);
      for (size_t i = 0; i < j.valid.size(); ++i) o[j.valid[i]] = std::move(r[i]);
    }
    for (auto& x : o) out.push_back(std::move(x));
  };
  for (int k = 0; k < std::min(L, nb); ++k) enqueue(k);
  for (int k = 0; k < nb; ++k) {
    start(k);
    if (k - J + 1 >= 0) finish(k - J + 1);
    if (k + L < nb) enqueue(k + L);
  }
  for (int k = std::max(0, nb - J + 1); k < nb; ++k) finish(k);
  // the call's stream sees every search and encoder complete (results are on the host)
  for (int s = 0; s < J; ++s) {
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 1], sst[s]));
    ZASR_HIP_CHECK(hipStreamWaitEvent(main_st, part_ev_[kMaxEnc + 1], 0));
  }
  if (E > 1) {
    ZASR_HIP_CHECK(hipEventRecord(part_ev_[kMaxEnc + 1], enc_st[1]));
    ZASR_HIP_CHECK(hipStreamWaitEvent(main_st, part_ev_[kMaxEnc + 1], 0));
  }
  st_ = stream_;
  return out;
}

std::vector<TokenResult> Engine::decode_features(const std::vector<const float*>& feats,
                                                 const std::vector<long>& frames, int beam) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  pin_reset(0);
  const int B = (int)feats.size();
  std::vector<int> valid, T;
  long tot = 0, tot_out = 0;
  for (int b = 0; b < B; ++b)
    if (frames[b] >= 9) {
      valid.push_back(b);
      T.push_back((int)frames[b]);
      tot += frames[b];
      tot_out += ((frames[b] - 7) / 2 + 1) / 2;
    }
  std::vector<TokenResult> out(B);
  if (valid.empty()) return out;
  float* d = ws<float>("feats", (size_t)tot * 80);
  long pos = 0;
  for (int b : valid) {
    ZASR_HIP_CHECK(hipMemcpyAsync(d + pos * 80, feats[b], (size_t)frames[b] * 80 * 4,
                                  hipMemcpyHostToDevice, st_));
    pos += frames[b];
  }
  float* enc = ws<float>("enc_out", (size_t)tot_out * model_.cfg.joiner_dim);
  std::vector<int> t_out;
  run_encoder(d, T, enc, t_out);
  std::vector<TokenResult> r = run_search(enc, t_out, beam);
  for (size_t i = 0; i < valid.size(); ++i) out[valid[i]] = std::move(r[i]);
  return out;
}

void Engine::fbank_host(const float* wav, long n, float* out) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  pin_reset(0);
  const long frames = n > 0 ? (n + 80) / 160 : 0;
  if (frames == 0) return;
  float* dw = ws<float>("fbh_wav", n);
  float* df = ws<float>("fbh_out", (size_t)frames * 80);
  ZASR_HIP_CHECK(hipMemcpyAsync(dw, wav, n * 4, hipMemcpyHostToDevice, st_));
  std::vector<int> fr;
  run_fbank(dw, {0}, {n}, df, fr);
  ZASR_HIP_CHECK(hipMemcpyAsync(out, df, (size_t)frames * 80 * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
}

void Engine::encode_host(const std::vector<const float*>& feats, const std::vector<long>& frames,
                         std::vector<float>& out, std::vector<int>& t_out) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  pin_reset(0);
  const int B = (int)feats.size();
  std::vector<int> T(B);
  long tot = 0, tot_out = 0;
  for (int b = 0; b < B; ++b) {
    ZASR_REQUIRE(frames[b] >= 9, "encoder needs >= 9 fbank frames per chunk");
    T[b] = (int)frames[b];
    tot += frames[b];
    tot_out += ((frames[b] - 7) / 2 + 1) / 2;
  }
  float* d = ws<float>("feats", (size_t)tot * 80);
  long pos = 0;
  for (int b = 0; b < B; ++b) {
    ZASR_HIP_CHECK(hipMemcpyAsync(d + pos * 80, feats[b], (size_t)frames[b] * 80 * 4,
                                  hipMemcpyHostToDevice, st_));
    pos += frames[b];
  }
  float* enc = ws<float>("enc_out", (size_t)tot_out * model_.cfg.joiner_dim);
  run_encoder(d, T, enc, t_out);
  out.resize((size_t)tot_out * model_.cfg.joiner_dim);
  ZASR_HIP_CHECK(hipMemcpyAsync(out.data(), enc, out.size() * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
}

std::vector<TokenResult> Engine::search_host(const std::vector<const float*>& enc,
                                             const std::vector<long>& t_out, int beam) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  pin_reset(0);
  const int B = (int)enc.size();
  const int D = model_.cfg.joiner_dim;
  long tot = 0;
  for (long t : t_out) tot += t;
  float* d = ws<float>("enc_in", (size_t)std::max<long>(tot, 1) * D);
  long pos = 0;
  std::vector<int> to(B);
  for (int b = 0; b < B; ++b) {
    to[b] = (int)t_out[b];
    if (t_out[b] > 0)
      ZASR_HIP_CHECK(hipMemcpyAsync(d + pos * D, enc[b], (size_t)t_out[b] * D * 4,
                                    hipMemcpyHostToDevice, st_));
    pos += t_out[b];
  }
  return run_search(d, to, beam);
}

}  // namespace zasr
