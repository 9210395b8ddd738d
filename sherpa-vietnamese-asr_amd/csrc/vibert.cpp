// ViBERT-capu engine: weight upload (fused QKV, fused label heads) and the forward pass.
#include "vibert.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "common.h"
#include "gemm.h"
#include "host_io.h"
#include "onnx_io.h"
#include "kernels.h"

namespace zasr {

template <class T>
T* VibertEngine::ws(const std::string& name, size_t count) {
  const size_t bytes = std::max<size_t>(count * sizeof(T), 256);
  auto& e = ws_[name];
  if (e.second < bytes) {
    if (e.first) {
      ZASR_HIP_CHECK(hipStreamSynchronize(st_));
      ZASR_HIP_CHECK(hipFree(e.first));
    }
    ZASR_HIP_CHECK(hipMalloc(&e.first, bytes + bytes / 8));
    e.second = bytes + bytes / 8;
  }
  return reinterpret_cast<T*>(e.first);
}

VibertEngine::VibertEngine(const std::string& dir, int device) : device_(device) {
  // vibert_config.json + vibert.safetensors, or the reference's vibert-capu.onnx (onnx_io.h)
  SafeTensors W;
  const Json j = Json::parse(load_stage_dir(dir, "vibert", W));
  H_ = (int)j.at("hidden_size").num;
  heads_ = (int)j.at("num_attention_heads").num;
  inter_ = (int)j.at("intermediate_size").num;
  labels_ = (int)j.at("num_labels").num;
  detect_ = (int)j.at("num_detect_classes").num;
  max_pos_ = (int)j.at("max_position_embeddings").num;
  eps_ = (float)j.at("layer_norm_eps").num;
  const int nl = (int)j.at("num_hidden_layers").num;
  ZASR_REQUIRE(heads_ > 0 && H_ % heads_ == 0 && H_ <= 1024 && H_ % 4 == 0,
               "ViBERT: hidden <= 1024, divisible by the head count");
  const int hd = H_ / heads_;
  ZASR_REQUIRE(hd == 16 || hd == 32 || hd == 64, "ViBERT: head dim 16, 32 or 64");
  ZASR_HIP_CHECK(hipSetDevice(device_));
  ZASR_HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
  auto dev = [&](const float* src, size_t n) {
    float* p = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(float)));
    ZASR_HIP_CHECK(hipMemcpy(p, src, n * sizeof(float), hipMemcpyHostToDevice));
    allocs_.push_back(p);
    return p;
  };
  auto get = [&](const std::string& n, size_t numel) {
    const HostTensor& t = W.get(n);
    ZASR_REQUIRE(t.numel == numel, "ViBERT: bad size of " + n);
    return t.data;
  };
  // rows of several [n_i][K] linears stacked into one GEMM weight
  auto stack = [&](const std::vector<std::pair<std::string, int>>& parts, int K) {
    std::vector<float> w, b;
    int N = 0;
    for (const auto& p : parts) {
      const float* pw = get(p.first + ".weight", (size_t)p.second * K);
      const float* pb = get(p.first + ".bias", (size_t)p.second);
      w.insert(w.end(), pw, pw + (size_t)p.second * K);
      b.insert(b.end(), pb, pb + p.second);
      N += p.second;
    }
    Lin l;
    l.w = dev(w.data(), w.size());
    l.b = dev(b.data(), b.size());
    l.N = N;
    l.K = K;
    return l;
  };
  const HostTensor& we = W.get("bert.embeddings.word_embeddings.weight");
  ZASR_REQUIRE(we.shape.size() == 2 && we.shape[1] == H_, "ViBERT: bad word embedding shape");
  word_ = dev(we.data, we.numel);
  vocab_ = (long)we.shape[0];
  pos_ = dev(get("bert.embeddings.position_embeddings.weight", (size_t)max_pos_ * H_), (size_t)max_pos_ * H_);
  const HostTensor& te = W.get("bert.embeddings.token_type_embeddings.weight");
  ZASR_REQUIRE(te.shape.size() == 2 && te.shape[1] == H_, "ViBERT: bad token type embedding shape");
  type_ = dev(te.data, te.numel);
  type_vocab_ = (long)te.shape[0];
  eln_g_ = dev(get("bert.embeddings.LayerNorm.weight", H_), H_);
  eln_b_ = dev(get("bert.embeddings.LayerNorm.bias", H_), H_);
  for (int i = 0; i < nl; ++i) {
    const std::string p = "bert.encoder.layer." + std::to_string(i) + ".";
    Layer L;
    L.qkv = stack({{p + "attention.self.query", H_}, {p + "attention.self.key", H_},
                   {p + "attention.self.value", H_}}, H_);
    L.ao = stack({{p + "attention.output.dense", H_}}, H_);
    L.inter = stack({{p + "intermediate.dense", inter_}}, H_);
    L.out = stack({{p + "output.dense", H_}}, inter_);
    L.ln1_g = dev(get(p + "attention.output.LayerNorm.weight", H_), H_);
    L.ln1_b = dev(get(p + "attention.output.LayerNorm.bias", H_), H_);
    L.ln2_g = dev(get(p + "output.LayerNorm.weight", H_), H_);
    L.ln2_b = dev(get(p + "output.LayerNorm.bias", H_), H_);
    layers_.push_back(L);
  }
  heads_lin_ = stack({{"classifier", labels_}, {"detector", detect_}}, H_);
  ZASR_HIP_CHECK(hipDeviceSynchronize());
}

VibertEngine::~VibertEngine() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(st_);
  for (void* p : allocs_) (void)hipFree(p);
  for (auto& kv : ws_)
    if (kv.second.first) (void)hipFree(kv.second.first);
  (void)hipStreamDestroy(st_);
}

void VibertEngine::gemm(const Lin& l, const float* A, int M, float* C, int epi) {
  GemmParams p{};
  p.A = A;
  p.lda = l.K;
  p.B = l.w;
  p.sbk = 1;
  p.sbn = l.K;
  p.C = C;
  p.ldc = l.N;
  p.bias = l.b;
  p.M = M;
  p.N = l.N;
  p.K = l.K;
  p.alpha = 1.f;
  p.max_M = M;
  gemm_f32(p, epi, ALOAD_DENSE, false, st_);
}

void VibertEngine::run_host(const long* ids, const long* am, const long* tt, const long* offs,
                            int B, int L, int W, float* logits, float* detect) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  ZASR_REQUIRE(B >= 0 && L >= 1 && L <= std::min(256, max_pos_) && W >= 1,
               "ViBERT: need 1 <= L <= 256 tokens and W >= 1 words");
  if (B == 0) return;
  const long R = (long)B * L;
  for (long i = 0; i < (long)B * W; ++i)
    ZASR_REQUIRE(offs[i] >= 0 && offs[i] < L, "ViBERT: input_offsets out of range");
  // the embedding kernel gathers rows by id: an id outside the tables would read out of
  // bounds on the device (onnxruntime's Gather raises instead)
  for (long i = 0; i < R; ++i) {
    ZASR_REQUIRE(ids[i] >= 0 && ids[i] < vocab_, "ViBERT: input_ids out of range");
    ZASR_REQUIRE(tt[i] >= 0 && tt[i] < type_vocab_, "ViBERT: token_type_ids out of range");
  }
  long* d_in = ws<long>("in", (size_t)R * 3 + (size_t)B * W);
  ZASR_HIP_CHECK(hipMemcpyAsync(d_in, ids, R * 8, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_in + R, am, R * 8, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_in + 2 * R, tt, R * 8, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_in + 3 * R, offs, (size_t)B * W * 8, hipMemcpyHostToDevice, st_));
  float* X = ws<float>("x", (size_t)R * H_);
  float* QKV = ws<float>("qkv", (size_t)R * 3 * H_);
  float* CTX = ws<float>("ctx", (size_t)R * H_);
  float* INT = ws<float>("int", (size_t)R * inter_);
  VibertEmbedArgs e{d_in, d_in + 2 * R, word_, pos_, type_, eln_g_, eln_b_, X, L, H_, eps_};
  launch_vibert_embed(e, R, st_);
  for (const Layer& ly : layers_) {
    gemm(ly.qkv, X, (int)R, QKV, EPI_NONE);
    VibertAttnArgs a{QKV, d_in + R, CTX, L, H_, 1.f / std::sqrt((float)(H_ / heads_))};
    launch_vibert_attention(a, B, heads_, st_);
    {
      GemmParams p{};
      p.A = CTX; p.lda = H_; p.B = ly.ao.w; p.sbk = 1; p.sbn = H_; p.C = X; p.ldc = H_;
      p.bias = ly.ao.b; p.M = (int)R; p.N = H_; p.K = H_; p.alpha = 1.f; p.max_M = (int)R;
      gemm_f32(p, EPI_RESADD, ALOAD_DENSE, false, st_);
    }
    launch_vibert_layernorm(X, R, H_, ly.ln1_g, ly.ln1_b, eps_, st_);
    gemm(ly.inter, X, (int)R, INT, EPI_GELU);
    {
      GemmParams p{};
      p.A = INT; p.lda = inter_; p.B = ly.out.w; p.sbk = 1; p.sbn = inter_; p.C = X; p.ldc = H_;
      p.bias = ly.out.b; p.M = (int)R; p.N = H_; p.K = inter_; p.alpha = 1.f; p.max_M = (int)R;
      gemm_f32(p, EPI_RESADD, ALOAD_DENSE, false, st_);
    }
    launch_vibert_layernorm(X, R, H_, ly.ln2_g, ly.ln2_b, eps_, st_);
  }
  const int BW = B * W;
  float* G = ws<float>("gather", (size_t)BW * H_);
  float* O = ws<float>("heads", (size_t)BW * heads_lin_.N);
  launch_vibert_gather(X, d_in + 3 * R, B, L, W, H_, G, st_);
  gemm(heads_lin_, G, BW, O, EPI_NONE);
  std::vector<float> h((size_t)BW * heads_lin_.N);
  ZASR_HIP_CHECK(hipMemcpyAsync(h.data(), O, h.size() * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
  for (int r = 0; r < BW; ++r) {
    std::memcpy(logits + (size_t)r * labels_, &h[(size_t)r * heads_lin_.N], labels_ * 4);
    std::memcpy(detect + (size_t)r * detect_, &h[(size_t)r * heads_lin_.N + labels_], detect_ * 4);
  }
}

}  // namespace zasr
