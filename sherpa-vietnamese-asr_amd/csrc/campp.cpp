// CAM++ speaker-embedding engine: weight folding / upload, fbank, forward.  See campp.h.
#include "campp.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "common.h"
#include "gemm.h"
#include "host_io.h"
#include "onnx_io.h"

namespace zasr {

namespace {
constexpr double kBnEps = 1e-5;

// eval BatchNorm as y = x * s + b; a BatchNorm the ONNX exporter already fused into the Conv
// before it (onnx_io.cpp load_campp_graph: "<bn>.fused_shift") is s = 1, b = the fused bias
void bn_fold(const SafeTensors& W, const std::string& p, int C, bool affine, std::vector<float>& s,
             std::vector<float>& b) {
  if (W.has(p + ".fused_shift")) {
    const HostTensor& f = W.get(p + ".fused_shift");
    ZASR_REQUIRE((int)f.numel == C, "CAM++: fused BN size mismatch for " + p);
    s.assign(C, 1.f);
    b.assign(f.data, f.data + C);
    return;
  }
  const HostTensor& m = W.get(p + ".running_mean");
  const HostTensor& v = W.get(p + ".running_var");
  ZASR_REQUIRE((int)m.numel == C && (int)v.numel == C, "CAM++: BN size mismatch for " + p);
  s.resize(C);
  b.resize(C);
  for (int c = 0; c < C; ++c) {
    const double g = affine ? W.get(p + ".weight").data[c] : 1.0;
    const double beta = affine ? W.get(p + ".bias").data[c] : 0.0;
    const double sc = g / std::sqrt((double)v.data[c] + kBnEps);
    s[c] = (float)sc;
    b[c] = (float)(beta - (double)m.data[c] * sc);
  }
}

std::vector<int> ints(const Json& j, const char* k, std::vector<int> dflt) {
  return j.has(k) ? j.at(k).as_int_vec() : dflt;
}
}  // namespace

template <class T>
T* CamppEngine::ws(const std::string& name, size_t count) {
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

CamppEngine::CamppEngine(const std::string& dir, int device) : device_(device) {
  // campp_config.json + campp.safetensors, or the reference's campplus_cn_en_common_200k.onnx
  SafeTensors W;
  const Json j = Json::parse(load_stage_dir(dir, "campp", W));
  if (j.has("feat_dim")) cfg_.feat_dim = (int)j.at("feat_dim").num;
  if (j.has("embedding_size")) cfg_.emb = (int)j.at("embedding_size").num;
  if (j.has("growth_rate")) cfg_.growth = (int)j.at("growth_rate").num;
  if (j.has("bn_size")) cfg_.bn_size = (int)j.at("bn_size").num;
  if (j.has("init_channels")) cfg_.init_ch = (int)j.at("init_channels").num;
  if (j.has("m_channels")) cfg_.m_ch = (int)j.at("m_channels").num;
  if (j.has("seg_len")) cfg_.seg_len = (int)j.at("seg_len").num;
  cfg_.head_blocks = ints(j, "head_blocks", cfg_.head_blocks);
  cfg_.block_layers = ints(j, "block_layers", cfg_.block_layers);
  cfg_.block_kernels = ints(j, "block_kernels", cfg_.block_kernels);
  cfg_.block_dil = ints(j, "block_dilations", cfg_.block_dil);
  ZASR_REQUIRE(cfg_.feat_dim == 80 && cfg_.m_ch == 32 && cfg_.growth == 32 && cfg_.bn_size == 4,
               "CAM++ kernels are specialised for feat_dim 80, m_channels 32, growth 32, bn_size 4");
  ZASR_HIP_CHECK(hipSetDevice(device_));
  ZASR_HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  st_ = stream_;
  auto dev = [&](const float* src, size_t n) {
    float* p = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(float)));
    ZASR_HIP_CHECK(hipMemcpy(p, src, n * sizeof(float), hipMemcpyHostToDevice));
    allocs_.push_back(p);
    return p;
  };
  auto devv = [&](const std::vector<float>& v) { return dev(v.data(), v.size()); };
  auto conv2 = [&](const std::string& w, const std::string& bn, int ci, int ks) {
    Conv2 c;
    const HostTensor& t = W.get(w);
    ZASR_REQUIRE(t.numel == (size_t)32 * ci * ks * ks, "CAM++: bad shape of " + w);
    c.w = dev(t.data, t.numel);
    if (ci == 32) {
      std::vector<float> pk(t.numel);
      campp_conv2d_permute_weights(t.data, ks, pk.data());
      c.wk = devv(pk);
    }
    std::vector<float> s, b;
    bn_fold(W, bn, 32, true, s, b);
    c.s = devv(s);
    c.b = devv(b);
    return c;
  };
  // a 1-D convolution [O][Cin][k] as an im2col GEMM weight [O][k * Cin + c], rows scaled
  // by a folded BN (scale / shift may be empty)
  auto lin = [&](const std::string& w, int O, int Cin, int k, const std::vector<float>& s,
                 const std::vector<float>& shift, const std::string& bias = "") {
    const HostTensor& t = W.get(w);
    ZASR_REQUIRE(t.numel == (size_t)O * Cin * k, "CAM++: bad shape of " + w);
    std::vector<float> p((size_t)O * Cin * k);
    for (int o = 0; o < O; ++o)
      for (int c = 0; c < Cin; ++c)
        for (int q = 0; q < k; ++q)
          p[(size_t)o * Cin * k + (size_t)q * Cin + c] =
              t.data[((size_t)o * Cin + c) * k + q] * (s.empty() ? 1.f : s[o]);
    Lin l;
    l.w = devv(p);
    l.N = O;
    l.K = Cin * k;
    if (!shift.empty()) {
      l.b = devv(shift);
    } else if (!bias.empty()) {
      l.b = dev(W.get(bias).data, O);
    }
    return l;
  };
  // ---- FCM head ----
  c1_ = conv2("head.conv1.weight", "head.bn1", 1, 3);
  for (size_t li = 0; li < cfg_.head_blocks.size(); ++li)
    for (int b = 0; b < cfg_.head_blocks[li]; ++b) {
      const std::string p = "head.layer" + std::to_string(li + 1) + "." + std::to_string(b) + ".";
      ResBlock r;
      r.stride = b == 0 ? 2 : 1;
      r.a = conv2(p + "conv1.weight", p + "bn1", 32, 3);
      r.b = conv2(p + "conv2.weight", p + "bn2", 32, 3);
      r.has_sc = W.has(p + "shortcut.0.weight");
      if (r.has_sc) r.sc = conv2(p + "shortcut.0.weight", p + "shortcut.1", 32, 1);
      res_.push_back(r);
    }
  c2_ = conv2("head.conv2.weight", "head.bn2", 32, 3);
  const int head_out = 32 * (cfg_.feat_dim / 8);
  {
    std::vector<float> s, b;
    bn_fold(W, "xvector.tdnn.nonlinear.batchnorm", cfg_.init_ch, true, s, b);
    tdnn_ = lin("xvector.tdnn.linear.weight", cfg_.init_ch, head_out, 5, s, b);
  }
  // ---- CAM dense TDNN blocks ----
  const int g = cfg_.growth, bnc = cfg_.bn_size * g;
  int c = cfg_.init_ch;
  for (size_t bi = 0; bi < cfg_.block_layers.size(); ++bi) {
    Block B;
    B.cin0 = c;
    B.cmax = c + cfg_.block_layers[bi] * g;
    B.dil = cfg_.block_dil[bi];
    B.k = cfg_.block_kernels[bi];
    for (int i = 0; i < cfg_.block_layers[bi]; ++i) {
      const std::string p = "xvector.block" + std::to_string(bi + 1) + ".tdnnd" + std::to_string(i + 1) + ".";
      DenseLayer L;
      L.cin = c + i * g;
      std::vector<float> s, b;
      bn_fold(W, p + "nonlinear1.batchnorm", L.cin, true, s, b);
      L.bn1_s = devv(s);
      L.bn1_b = devv(b);
      std::vector<float> s2, b2;
      bn_fold(W, p + "nonlinear2.batchnorm", bnc, true, s2, b2);
      L.l1 = lin(p + "linear1.weight", bnc, L.cin, 1, s2, b2);
      L.local = lin(p + "cam_layer.linear_local.weight", g, bnc, B.k, {}, {});
      L.m1w = dev(W.get(p + "cam_layer.linear1.weight").data, (size_t)(bnc / 2) * bnc);
      L.m1b = dev(W.get(p + "cam_layer.linear1.bias").data, bnc / 2);
      L.m2w = dev(W.get(p + "cam_layer.linear2.weight").data, (size_t)g * (bnc / 2));
      L.m2b = dev(W.get(p + "cam_layer.linear2.bias").data, g);
      B.layers.push_back(L);
    }
    std::vector<float> s, b;
    const std::string tp = "xvector.transit" + std::to_string(bi + 1) + ".";
    bn_fold(W, tp + "nonlinear.batchnorm", B.cmax, true, s, b);
    B.tr_s = devv(s);
    B.tr_b = devv(b);
    B.transit = lin(tp + "linear.weight", B.cmax / 2, B.cmax, 1, {}, {});
    blocks_.push_back(B);
    c = B.cmax / 2;
  }
  {
    std::vector<float> s, b;
    bn_fold(W, "xvector.out_nonlinear.batchnorm", c, true, s, b);
    out_s_ = devv(s);
    out_b_ = devv(b);
    std::vector<float> s2, b2;
    bn_fold(W, "xvector.dense.nonlinear.batchnorm", cfg_.emb, false, s2, b2);
    dense_ = lin("xvector.dense.linear.weight", cfg_.emb, 2 * c, 1, s2, b2);
  }
  // ---- fbank tables: kaldi mel bank 20 Hz .. Nyquist (high_freq 0), povey window ----
  {
    std::vector<double> tw(512);
    for (int i = 0; i < 256; ++i) {
      const double a = -2.0 * M_PI * i / 512.0;
      tw[2 * i] = std::cos(a);
      tw[2 * i + 1] = std::sin(a);
    }
    ZASR_HIP_CHECK(hipMalloc(&d_twiddle_, 512 * sizeof(double)));
    ZASR_HIP_CHECK(hipMemcpy(d_twiddle_, tw.data(), 512 * sizeof(double), hipMemcpyHostToDevice));
    std::vector<float> win(400);
    for (int i = 0; i < 400; ++i) win[i] = (float)std::pow(0.5 - 0.5 * std::cos(2.0 * M_PI * i / 399.0), 0.85);
    d_window_ = dev(win.data(), 400);
    auto mel = [](double f) { return 1127.0 * std::log(1.0 + f / 700.0); };
    const double mlo = mel(20.0), mhi = mel(8000.0), delta = (mhi - mlo) / 81.0;
    std::vector<int> meta(240);
    std::vector<float> wts;
    for (int b = 0; b < 80; ++b) {
      const double l = mlo + b * delta, ce = mlo + (b + 1) * delta, r = mlo + (b + 2) * delta;
      int st = -1, en = -1;
      std::vector<float> row(256, 0.f);
      for (int i = 0; i < 256; ++i) {
        const double m = mel(31.25 * i);
        if (m > l && m < r) {
          row[i] = (float)(m <= ce ? (m - l) / (ce - l) : (r - m) / (r - ce));
          if (st < 0) st = i;
          en = i;
        }
      }
      if (st < 0) st = en = 0;
      meta[b] = st;
      meta[80 + b] = en - st + 1;
      meta[160 + b] = (int)wts.size();
      for (int i = st; i <= en; ++i) wts.push_back(row[i]);
    }
    ZASR_HIP_CHECK(hipMalloc(&d_mel_meta_, 240 * sizeof(int)));
    ZASR_HIP_CHECK(hipMemcpy(d_mel_meta_, meta.data(), 240 * sizeof(int), hipMemcpyHostToDevice));
    d_mel_w_ = dev(wts.data(), wts.size());
  }
  ZASR_HIP_CHECK(hipDeviceSynchronize());
}

CamppEngine::~CamppEngine() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(stream_);
  for (void* p : allocs_) (void)hipFree(p);
  for (auto& kv : ws_)
    if (kv.second.first) (void)hipFree(kv.second.first);
  if (d_twiddle_) (void)hipFree(d_twiddle_);
  if (d_mel_meta_) (void)hipFree(d_mel_meta_);
  (void)hipStreamDestroy(stream_);
}

void CamppEngine::gemm(const Lin& l, const float* A, int lda, int M, float* C, int ldc, int epi,
                       const float* aux, int ldaux, int aload, const float* a_scale,
                       const float* a_shift, const GemmIm2col1d* i2c) {
  GemmParams p{};
  p.A = A;
  p.lda = lda;
  p.B = l.w;
  p.sbk = 1;
  p.sbn = l.K;
  p.C = C;
  p.ldc = ldc;
  p.bias = l.b;
  p.aux = aux;
  p.ldaux = ldaux;
  p.M = M;
  p.N = l.N;
  p.K = l.K;
  p.alpha = 1.f;
  p.max_M = M;
  p.a_scale = a_scale;
  p.a_shift = a_shift;
  if (i2c) p.i2c = *i2c;
  gemm_f32(p, epi, aload, false, st_);
}

void CamppEngine::fbank_host(const float* wav, long n, std::vector<float>& out) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  const long frames = n >= 400 ? 1 + (n - 400) / 160 : 0;
  out.assign((size_t)frames * 80, 0.f);
  if (frames == 0) return;
  float* dw = ws<float>("fb_wav", n);
  float* df = ws<float>("fb_out", (size_t)frames * 80);
  long* doff = ws<long>("fb_off", 1);
  int* dmeta = ws<int>("fb_meta", 3);
  const long zero = 0;
  const int meta[3] = {(int)n, 0, (int)frames};
  ZASR_HIP_CHECK(hipMemcpyAsync(dw, wav, n * 4, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(doff, &zero, sizeof(long), hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(dmeta, meta, sizeof(meta), hipMemcpyHostToDevice, st_));
  FbankTables t{d_twiddle_, d_window_, d_mel_meta_, d_mel_meta_ + 80, d_mel_meta_ + 160, d_mel_w_};
  launch_fbank(dw, doff, dmeta, dmeta + 1, 1, (int)frames, t, df, st_, true);
  launch_campp_cmvn(df, dmeta + 1, 1, st_);
  ZASR_HIP_CHECK(hipMemcpyAsync(out.data(), df, out.size() * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
}

long CamppEngine::windows_device(const float* d_wav, const long* reg_off, const long* reg_len,
                                 int nreg, int wf, int sf, float* d_feats, long max_windows,
                                 int* win_region, int* win_first, int* win_frames,
                                 hipStream_t st) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = st ? st : stream_;
  ZASR_REQUIRE(wf >= 1 && sf >= 1, "CAM++ windows: window and step must be >= 1 frame");
  // regions that yield windows (>= 10 fbank frames, :547-556), their packed fbank rows and
  // the window plan (:558-582)
  std::vector<long> woff;
  std::vector<int> ns, fr_off{0}, wrow, wn;
  long nwin = 0;
  for (int r = 0; r < nreg; ++r) {
    const long n = reg_len[r];
    ZASR_REQUIRE(n >= 0 && n <= INT32_MAX, "CAM++ windows: region length out of range");
    const long frames = n >= 400 ? 1 + (n - 400) / 160 : 0;
    if (frames < 10) continue;
    const int base = fr_off.back();
    auto add = [&](long first, long cnt) {
      ZASR_REQUIRE(nwin < max_windows, "CAM++ windows: more windows than max_windows");
      win_region[nwin] = r;
      win_first[nwin] = (int)first;
      win_frames[nwin] = (int)cnt;
      wrow.push_back(base + (int)first);
      wn.push_back((int)cnt);
      ++nwin;
    };
    if (frames < wf) {
      add(0, frames);
    } else {
      long pos = 0;
      for (; pos + wf < frames; pos += sf) add(pos, wf);  // strict < (:565)
      add(std::max<long>(0, frames - wf), wf);            // tail pulled back (:572-577)
    }
    woff.push_back(reg_off[r]);
    ns.push_back((int)n);
    ZASR_REQUIRE((long)base + frames <= INT32_MAX, "CAM++ windows: too many fbank frames");
    fr_off.push_back(base + (int)frames);
  }
  const int nv = (int)ns.size();
  if (nwin == 0) return 0;
  const int total = fr_off.back();
  long* d_woff = ws<long>("wd_woff", nv);
  int* d_ns = ws<int>("wd_ns", nv);
  int* d_fo = ws<int>("wd_fo", nv + 1);
  int* d_wrow = ws<int>("wd_wrow", nwin);
  int* d_wn = ws<int>("wd_wn", nwin);
  float* rows = ws<float>("wd_rows", (size_t)total * 80);
  // pageable sources: HIP stages each copy before returning
  ZASR_HIP_CHECK(hipMemcpyAsync(d_woff, woff.data(), nv * sizeof(long), hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_ns, ns.data(), nv * sizeof(int), hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_fo, fr_off.data(), (nv + 1) * sizeof(int), hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_wrow, wrow.data(), nwin * sizeof(int), hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_wn, wn.data(), nwin * sizeof(int), hipMemcpyHostToDevice, st_));
  FbankTables t{d_twiddle_, d_window_, d_mel_meta_, d_mel_meta_ + 80, d_mel_meta_ + 160, d_mel_w_};
  launch_fbank(d_wav, d_woff, d_ns, d_fo, nv, total, t, rows, st_, true);
  launch_campp_cmvn(rows, d_fo, nv, st_);
  launch_campp_gather(rows, d_wrow, d_wn, (int)nwin, wf, d_feats, st_);
  return nwin;
}

void CamppEngine::embed_device(const float* d_feats, int N, int T, float* d_out, hipStream_t st) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = st ? st : stream_;
  if (N <= 0) return;
  ZASR_REQUIRE(T >= 1, "CAM++: T must be >= 1");
  // ---- FCM head, [N][32][F][T] ----
  auto conv = [&](const Conv2& c, const float* x, int ci, int fi, int sf, int ks, const float* res,
                  bool relu, float* y, bool tdnn, bool in_tf) {
    CamppConv2d a{};
    a.x = x;
    a.w = c.w;
    a.wk = c.wk;
    a.scale = c.s;
    a.shift = c.b;
    a.res = res;
    a.y = y;
    a.n = N;
    a.ci = ci;
    a.fi = fi;
    a.fo = (fi - 1) / sf + 1;
    a.T = T;
    a.sf = sf;
    a.relu = relu;
    a.tdnn_out = tdnn;
    a.in_tf = in_tf;
    launch_campp_conv2d(a, ks, st_);
    return a.fo;
  };
  int F = cfg_.feat_dim;
  const size_t plane = (size_t)N * 32 * F * T;
  float* x = ws<float>("h_x", plane);
  float* t1 = ws<float>("h_t1", plane);
  float* sc = ws<float>("h_sc", plane);
  float* y = ws<float>("h_y", plane);
  conv(c1_, d_feats, 1, F, 1, 3, nullptr, true, x, false, true);
  for (const ResBlock& r : res_) {
    const int Fo = conv(r.a, x, 32, F, r.stride, 3, nullptr, true, t1, false, false);
    const float* shortcut = x;
    if (r.has_sc) {
      conv(r.sc, x, 32, F, r.stride, 1, nullptr, false, sc, false, false);
      shortcut = sc;
    }
    F = Fo;
    conv(r.b, t1, 32, F, 1, 3, shortcut, true, y, false, false);
    std::swap(x, y);
  }
  const int Fh = (F - 1) / 2 + 1;
  const int head_out = 32 * Fh;
  float* h = ws<float>("h_out", (size_t)N * T * head_out);
  conv(c2_, x, 32, F, 2, 3, nullptr, true, h, true, false);
  // ---- TDNN (k 5, stride 2, pad 2) ----
  const int T2 = (T - 1) / 2 + 1;
  const int R = N * T2;
  // the im2col of both 1-D convolutions and the BN-ReLU in front of the dense layers' 1 x 1
  // and transit projections happen in the GEMM's A loader (ALOAD_IM2COL1D / ALOAD_BNRELU)
  float* X = ws<float>("blk0", (size_t)R * blocks_[0].cmax);
  const GemmIm2col1d tdnn_i2c{T, T2, head_out, 2, 1, 2};
  gemm(tdnn_, h, head_out, R, X, blocks_[0].cmax, EPI_RELU, nullptr, 0, ALOAD_IM2COL1D, nullptr,
       nullptr, &tdnn_i2c);
  // ---- dense blocks ----
  const int bnc = cfg_.bn_size * cfg_.growth;
  float* H2 = ws<float>("h2", (size_t)R * bnc);
  float* mexp = ws<float>("mexp", (size_t)R * cfg_.growth);
  for (size_t bi = 0; bi < blocks_.size(); ++bi) {
    const Block& B = blocks_[bi];
    for (const DenseLayer& L : B.layers) {
      gemm(L.l1, X, B.cmax, R, H2, bnc, EPI_RELU, nullptr, 0, ALOAD_BNRELU, L.bn1_s, L.bn1_b);
      CamppCamMask m{H2, L.m1w, L.m1b, L.m2w, L.m2b, mexp, N, T2, cfg_.seg_len};
      launch_campp_cam_mask(m, st_);
      const int pad = (B.k - 1) / 2 * B.dil;
      const GemmIm2col1d i2c{T2, T2, bnc, 1, B.dil, pad};
      gemm(L.local, H2, bnc, R, X + L.cin, B.cmax, EPI_MULAUX, mexp, cfg_.growth, ALOAD_IM2COL1D,
           nullptr, nullptr, &i2c);
    }
    const int next_ld = bi + 1 < blocks_.size() ? blocks_[bi + 1].cmax : B.cmax / 2;
    float* Xn = ws<float>("blk" + std::to_string(bi + 1), (size_t)R * next_ld);
    gemm(B.transit, X, B.cmax, R, Xn, next_ld, EPI_NONE, nullptr, 0, ALOAD_BNRELU, B.tr_s, B.tr_b);
    X = Xn;
  }
  // ---- BN-ReLU + statistics pooling + dense (affine-free BN folded) ----
  const int C = blocks_.back().cmax / 2;
  float* P = ws<float>("pool", (size_t)N * 2 * C);
  launch_campp_stats(X, N, T2, C, out_s_, out_b_, P, st_);
  gemm(dense_, P, 2 * C, N, d_out, cfg_.emb, EPI_NONE);
}

void CamppEngine::embed_host(const float* feats, int N, int T, float* out) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  st_ = stream_;
  if (N <= 0) return;
  float* df = ws<float>("in_feats", (size_t)N * T * cfg_.feat_dim);
  float* dout = ws<float>("in_out", (size_t)N * cfg_.emb);
  ZASR_HIP_CHECK(hipMemcpyAsync(df, feats, (size_t)N * T * cfg_.feat_dim * 4, hipMemcpyHostToDevice, st_));
  embed_device(df, N, T, dout, stream_);
  ZASR_HIP_CHECK(hipMemcpyAsync(out, dout, (size_t)N * cfg_.emb * 4, hipMemcpyDeviceToHost, stream_));
  ZASR_HIP_CHECK(hipStreamSynchronize(stream_));
}

}  // namespace zasr
