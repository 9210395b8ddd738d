// Silero VAD engine: weight layout for the GEMM formulation and the batched forward pass.
#include "vad.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "gemm.h"
#include "host_io.h"
#include "onnx_io.h"
#include "kernels.h"

namespace zasr {

namespace {
constexpr int VW = 512, VIN = 576, VFR = 4, VFL = 256, VH = 128;
}

template <class T>
T* VadEngine::ws(const std::string& name, size_t count) {
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

VadEngine::VadEngine(const std::string& dir, int device) : device_(device) {
  // silero_config.json + silero_vad.safetensors, or the reference's silero_vad_16k_op15.onnx
  SafeTensors W;
  const Json j = Json::parse(load_stage_dir(dir, "silero", W));
  ZASR_REQUIRE(j.at("window").as_int() == VW && j.at("context").as_int() == VIN - VW &&
                   j.at("filter_length").as_int() == VFL && j.at("hop").as_int() == 128 &&
                   j.at("hidden").as_int() == VH,
               "Silero VAD: only the 16 kHz v5 shape (window 512, context 64, STFT 256/128, LSTM 128)");
  const std::vector<int> ch = j.at("enc_channels").as_int_vec(), sd = j.at("enc_strides").as_int_vec();
  ZASR_REQUIRE(ch.size() == sd.size() && !ch.empty() && ch.back() == VH, "Silero VAD: bad encoder config");
  ZASR_HIP_CHECK(hipSetDevice(device_));
  ZASR_HIP_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
  {
    hipDeviceProp_t prop;
    ZASR_HIP_CHECK(hipGetDeviceProperties(&prop, device_));
    cus_ = std::max(1, prop.multiProcessorCount);
    const char* e = std::getenv("ZASR_VAD_PIT");
    pit_ = !(e && e[0] == '0');
  }
  auto dev = [&](const float* src, size_t n) {
    float* p = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(float)));
    ZASR_HIP_CHECK(hipMemcpy(p, src, n * sizeof(float), hipMemcpyHostToDevice));
    allocs_.push_back(p);
    return p;
  };
  auto get = [&](const std::string& n, size_t numel) {
    const HostTensor& t = W.get("_model." + n);
    ZASR_REQUIRE(t.numel == numel, "Silero VAD: bad size of " + n);
    return t.data;
  };
  // STFT basis [2 bins][1][256] -> GEMM weight [N = 2 bins padded to 4][K = 256]
  const int nb2 = 2 * bins_, nbp = (nb2 + 3) / 4 * 4;
  {
    std::vector<float> w((size_t)nbp * VFL, 0.f);
    std::memcpy(w.data(), get("stft.forward_basis_buffer", (size_t)nb2 * VFL), (size_t)nb2 * VFL * 4);
    stft_.w = dev(w.data(), w.size());
    stft_.N = nbp;
    stft_.K = VFL;
  }
  // Conv1d(k 3) weights [co][ci][3] -> im2col GEMM weights [co][Kp], column k * ci + c
  int cin = bins_;
  for (size_t i = 0; i < ch.size(); ++i) {
    const std::string p = "encoder." + std::to_string(i) + ".reparam_conv.";
    const int co = ch[i], K = 3 * cin, Kp = (K + 3) / 4 * 4;
    const float* src = get(p + "weight", (size_t)co * cin * 3);
    std::vector<float> w((size_t)co * Kp, 0.f);
    for (int o = 0; o < co; ++o)
      for (int c = 0; c < cin; ++c)
        for (int k = 0; k < 3; ++k) w[(size_t)o * Kp + k * cin + c] = src[((size_t)o * cin + c) * 3 + k];
    Lin l;
    l.w = dev(w.data(), w.size());
    l.b = dev(get(p + "bias", co), co);
    l.N = co;
    l.K = Kp;
    conv_.push_back(l);
    cin_.push_back(cin);
    stride_.push_back(sd[i]);
    if (i == 0) kp1_ = Kp;
    cin = co;
  }
  ih_.w = dev(get("decoder.rnn.weight_ih", (size_t)4 * VH * VH), (size_t)4 * VH * VH);
  ih_.b = dev(get("decoder.rnn.bias_ih", 4 * VH), 4 * VH);
  ih_.N = 4 * VH;
  ih_.K = VH;
  whh_ = dev(get("decoder.rnn.weight_hh", (size_t)4 * VH * VH), (size_t)4 * VH * VH);
  bhh_ = dev(get("decoder.rnn.bias_hh", 4 * VH), 4 * VH);
  wd_ = dev(get("decoder.decoder.2.weight", VH), VH);
  bd_ = get("decoder.decoder.2.bias", 1)[0];
  ZASR_HIP_CHECK(hipDeviceSynchronize());
}

VadEngine::~VadEngine() {
  (void)hipSetDevice(device_);
  (void)hipStreamSynchronize(st_);
  for (void* p : allocs_) (void)hipFree(p);
  for (auto& kv : ws_)
    if (kv.second.first) (void)hipFree(kv.second.first);
  (void)hipStreamDestroy(st_);
}

void VadEngine::gemm(const Lin& l, const float* A, long M, float* C, int ldc, int epi) {
  ZASR_REQUIRE(M < (1L << 31), "Silero VAD: too many windows in one call");
  GemmParams p{};
  p.A = A;
  p.lda = l.K;
  p.B = l.w;
  p.sbk = 1;
  p.sbn = l.K;
  p.C = C;
  p.ldc = ldc;
  p.bias = l.b;
  p.M = (int)M;
  p.N = l.N;
  p.K = l.K;
  p.alpha = 1.f;
  p.max_M = (int)M;
  gemm_f32(p, epi, ALOAD_DENSE, false, st_);
}

float* VadEngine::encode(long n) {
  float* F = ws<float>("frames", (size_t)n * VFR * VFL);
  float* S = ws<float>("stft", (size_t)n * VFR * stft_.N);
  gemm(stft_, F, n * VFR, S, stft_.N, EPI_NONE);
  float* A = ws<float>("im2col", (size_t)n * VFR * kp1_);
  launch_vad_mag_im2col(S, stft_.N, bins_, kp1_, n, A, st_);
  float* Y = ws<float>("y0", (size_t)n * VFR * conv_[0].N);
  gemm(conv_[0], A, n * VFR, Y, conv_[0].N, EPI_RELU);
  int T = (VFR + 2 - 3) / stride_[0] + 1;
  for (size_t i = 1; i < conv_.size(); ++i) {
    const int To = (T + 2 - 3) / stride_[i] + 1;
    float* A2 = ws<float>("im2col", (size_t)n * To * conv_[i].K);
    launch_vad_im2col(Y, n, T, cin_[i], stride_[i], To, A2, st_);
    float* Y2 = ws<float>(i & 1 ? "y1" : "y0", (size_t)n * To * conv_[i].N);
    gemm(conv_[i], A2, n * To, Y2, conv_[i].N, EPI_RELU);
    Y = Y2;
    T = To;
  }
  ZASR_REQUIRE(T == 1, "Silero VAD: encoder must reduce the 4 STFT frames to 1");
  float* GX = ws<float>("gx", (size_t)n * 4 * VH);
  gemm(ih_, Y, n, GX, 4 * VH, EPI_NONE);
  return GX;
}

void VadEngine::probs_device(const float* d_audio, const long* off, const long* len, int n_files,
                             bool auto_boost, float* d_probs, hipStream_t user_stream) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  ZASR_REQUIRE(n_files >= 0, "Silero VAD: negative file count");
  std::vector<long> meta((size_t)3 * n_files);  // off | len | first window
  long nw = 0;
  std::vector<long> sw_start;
  std::vector<int> sw_count;
  for (int i = 0; i < n_files; ++i) {
    ZASR_REQUIRE(len[i] >= 0 && off[i] >= 0, "Silero VAD: negative offset / length");
    meta[i] = off[i];
    meta[n_files + i] = len[i];
    meta[2 * n_files + i] = nw;
    const long w = len[i] / VW;
    if (w > 0) {
      sw_start.push_back(nw);
      sw_count.push_back((int)w);
    }
    nw += w;
  }
  if (nw == 0) return;
  if (user_stream) {  // order after the caller's producer of d_audio
    hipEvent_t ev;
    ZASR_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ZASR_HIP_CHECK(hipEventRecord(ev, user_stream));
    ZASR_HIP_CHECK(hipStreamWaitEvent(st_, ev, 0));
    ZASR_HIP_CHECK(hipEventDestroy(ev));
  }
  long* d_meta = ws<long>("meta", meta.size());
  unsigned* d_mx = ws<unsigned>("maxabs", (size_t)n_files);
  ZASR_HIP_CHECK(hipMemcpyAsync(d_meta, meta.data(), meta.size() * 8, hipMemcpyHostToDevice, st_));
  if (auto_boost) {
    ZASR_HIP_CHECK(hipMemsetAsync(d_mx, 0, (size_t)n_files * 4, st_));
    launch_vad_maxabs(d_audio, d_meta, d_meta + n_files, n_files, d_mx, st_);
  }
  VadFramesArgs fa{};
  fa.audio = d_audio;
  fa.off = d_meta;
  fa.win_start = d_meta + 2 * n_files;
  fa.maxabs = auto_boost ? d_mx : nullptr;
  fa.frames = ws<float>("frames", (size_t)nw * VFR * VFL);
  fa.n_files = n_files;
  launch_vad_frames(fa, nw, st_);
  recurrence(encode(nw), sw_start, sw_count, nw, d_probs);
  if (user_stream) {
    hipEvent_t ev;
    ZASR_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    ZASR_HIP_CHECK(hipEventRecord(ev, st_));
    ZASR_HIP_CHECK(hipStreamWaitEvent(user_stream, ev, 0));
    ZASR_HIP_CHECK(hipEventDestroy(ev));
  } else {
    ZASR_HIP_CHECK(hipStreamSynchronize(st_));
  }
}

// The LSTM over every file's windows.  A file's windows are cut into segments decoded in
// parallel (about one workgroup per CU over the whole job); segment k > 0 first guesses its
// start state by running up to 256 warm-up windows from zeros (the recurrence is contractive:
// a state error of O(10) decays to O(1e-8) in ~200 windows on speech).  The host then checks
// the chain: segment k is accepted if the state it started from matches segment k-1's end
// state to kStateTol (relative, per element) -- the rounding-noise level at which a sequential
// run already differs from one with another summation order.  From the first mismatch on,
// segments rerun from their predecessor's end state, which validates at least one more
// segment per pass; after kMaxPass passes the unverified rest of a file runs as one sequential
// segment.  ZASR_VAD_PIT=0 turns this off (one sequential workgroup per file).
void VadEngine::recurrence(const float* GX, const std::vector<long>& f_start,
                           const std::vector<int>& f_count, long nw, float* d_probs) {
  constexpr int kMinSeg = 128, kWarm = 256, kMaxPass = 6, S2 = 2 * VH;
  constexpr float kStateTol = 1e-6f;
  struct Seg {
    long start;
    int count, warm;
  };
  std::vector<Seg> seg;
  std::vector<int> f_first;  // first segment of each file
  const double target = cus_;
  for (size_t f = 0; f < f_start.size(); ++f) {
    const int w = f_count[f];
    int K = (int)std::llround(target * (double)w / (double)nw);
    K = std::max(1, std::min(K, w / kMinSeg));
    if (!pit_) K = 1;
    f_first.push_back((int)seg.size());
    for (int k = 0; k < K; ++k) {
      const long a = (long)w * k / K, b = (long)w * (k + 1) / K;
      seg.push_back({f_start[f] + a, (int)(b - a), (int)std::min<long>(kWarm, a)});
    }
  }
  f_first.push_back((int)seg.size());
  const int NS = (int)seg.size();
  std::vector<float> S((size_t)NS * S2, 0.f), E((size_t)NS * S2, 0.f);
  long* d_start = ws<long>("seg_start", (size_t)NS);
  int* d_cnt = ws<int>("seg_count", (size_t)NS);
  int* d_warm = ws<int>("seg_warm", (size_t)NS);
  float* d_init = ws<float>("seg_init", (size_t)NS * S2);
  float* d_s = ws<float>("seg_s", (size_t)NS * S2);
  float* d_e = ws<float>("seg_e", (size_t)NS * S2);
  VadLstmArgs la{};
  la.gx = GX;
  la.whh = whh_;
  la.bhh = bhh_;
  la.wd = wd_;
  la.bd = bd_;
  la.seg_start = d_start;
  la.seg_count = d_cnt;
  la.probs = d_probs;
  auto launch = [&](const std::vector<long>& st, const std::vector<int>& cnt,
                    const std::vector<int>* warm, const std::vector<float>* init, bool want_s) {
    const int n = (int)st.size();
    ZASR_HIP_CHECK(hipMemcpyAsync(d_start, st.data(), (size_t)n * 8, hipMemcpyHostToDevice, st_));
    ZASR_HIP_CHECK(hipMemcpyAsync(d_cnt, cnt.data(), (size_t)n * 4, hipMemcpyHostToDevice, st_));
    la.seg_warm = nullptr;
    if (warm) {
      ZASR_HIP_CHECK(hipMemcpyAsync(d_warm, warm->data(), (size_t)n * 4, hipMemcpyHostToDevice, st_));
      la.seg_warm = d_warm;
    }
    la.init = nullptr;
    if (init) {
      ZASR_HIP_CHECK(hipMemcpyAsync(d_init, init->data(), (size_t)n * S2 * 4, hipMemcpyHostToDevice, st_));
      la.init = d_init;
    }
    la.s_out = want_s ? d_s : nullptr;
    la.e_out = d_e;
    launch_vad_lstm(la, n, st_);
  };
  // pass 0: every segment, warm-up guesses
  {
    std::vector<long> st(NS);
    std::vector<int> cnt(NS), warm(NS);
    for (int i = 0; i < NS; ++i) {
      st[i] = seg[i].start;
      cnt[i] = seg[i].count;
      warm[i] = seg[i].warm;
    }
    launch(st, cnt, &warm, nullptr, true);
    if (NS == (int)f_start.size()) {  // one segment per file: exact, nothing to verify
      last_passes_ = 1;
      return;
    }
    ZASR_HIP_CHECK(hipMemcpyAsync(S.data(), d_s, S.size() * 4, hipMemcpyDeviceToHost, st_));
    ZASR_HIP_CHECK(hipMemcpyAsync(E.data(), d_e, E.size() * 4, hipMemcpyDeviceToHost, st_));
    ZASR_HIP_CHECK(hipStreamSynchronize(st_));
  }
  const size_t nf = f_start.size();
  std::vector<int> k0(nf);  // first unverified segment of each file (global index)
  // continuity at a segment boundary: the start state a segment ran from vs its predecessor's
  // end state, to the rounding-noise level of the recurrence (two runs whose states once
  // differed keep differing by a few ulp for ~10^3 steps before they coincide bit for bit)
  auto same = [&](const float* a, const float* b) {
    for (int i = 0; i < S2; ++i) {
      const float d = std::fabs(a[i] - b[i]);
      if (!(d <= kStateTol * (1.f + std::fabs(b[i])))) return false;
    }
    return true;
  };
  auto verify = [&](size_t f, int from) {
    int k = std::max(from, f_first[f] + 1);
    for (; k < f_first[f + 1]; ++k)
      if (!same(&S[(size_t)k * S2], &E[(size_t)(k - 1) * S2])) break;
    return k;
  };
  for (size_t f = 0; f < nf; ++f) k0[f] = verify(f, f_first[f] + 1);
  int pass = 1;
  for (;; ++pass) {
    std::vector<long> st;
    std::vector<int> cnt, idx;
    std::vector<float> init;
    const bool last = pass >= kMaxPass;
    for (size_t f = 0; f < nf; ++f) {
      if (k0[f] >= f_first[f + 1]) continue;
      const int k = k0[f];
      if (last) {  // the rest of the file as one sequential segment from the exact state
        st.push_back(seg[k].start);
        cnt.push_back((int)(seg[f_first[f + 1] - 1].start + seg[f_first[f + 1] - 1].count - seg[k].start));
        idx.push_back(-1);
        init.insert(init.end(), &E[(size_t)(k - 1) * S2], &E[(size_t)k * S2]);
        continue;
      }
      for (int i = k; i < f_first[f + 1]; ++i) {
        st.push_back(seg[i].start);
        cnt.push_back(seg[i].count);
        idx.push_back(i);
        init.insert(init.end(), &E[(size_t)(i - 1) * S2], &E[(size_t)i * S2]);
      }
    }
    if (st.empty()) break;
    launch(st, cnt, nullptr, &init, false);
    if (last) {
      ++pass;
      break;
    }
    std::vector<float> e((size_t)st.size() * S2);
    ZASR_HIP_CHECK(hipMemcpyAsync(e.data(), d_e, e.size() * 4, hipMemcpyDeviceToHost, st_));
    ZASR_HIP_CHECK(hipStreamSynchronize(st_));
    for (size_t i = 0; i < idx.size(); ++i) {
      std::memcpy(&S[(size_t)idx[i] * S2], &init[i * S2], S2 * 4);
      std::memcpy(&E[(size_t)idx[i] * S2], &e[i * S2], S2 * 4);
    }
    for (size_t f = 0; f < nf; ++f)
      if (k0[f] < f_first[f + 1]) k0[f] = verify(f, k0[f] + 1);
  }
  last_passes_ = pass;
}

void VadEngine::probs_host(const float* audio, const long* off, const long* len, int n_files,
                           bool auto_boost, float* probs) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  long total = 0, nw = 0;
  for (int i = 0; i < n_files; ++i) {
    ZASR_REQUIRE(len[i] >= 0 && off[i] >= 0, "Silero VAD: negative offset / length");
    total = std::max(total, off[i] + len[i]);
    nw += len[i] / VW;
  }
  if (nw == 0) return;
  float* d_audio = ws<float>("audio", (size_t)total);
  float* d_probs = ws<float>("probs", (size_t)nw);
  ZASR_HIP_CHECK(hipMemcpyAsync(d_audio, audio, (size_t)total * 4, hipMemcpyHostToDevice, st_));
  probs_device(d_audio, off, len, n_files, auto_boost, d_probs, nullptr);
  ZASR_HIP_CHECK(hipMemcpyAsync(probs, d_probs, (size_t)nw * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
}

void VadEngine::window_host(const float* input, const float* state, int n, float* prob,
                            float* state_out) {
  ZASR_HIP_CHECK(hipSetDevice(device_));
  if (n <= 0) return;
  constexpr int S2 = 2 * VH;
  float* d_in = ws<float>("rows", (size_t)n * VIN);
  float* d_init = ws<float>("w_init", (size_t)n * S2);
  float* d_e = ws<float>("w_e", (size_t)n * S2);
  long* d_ws = ws<long>("w_start", (size_t)n);
  int* d_wc = ws<int>("w_count", (size_t)n);
  float* d_p = ws<float>("w_probs", (size_t)n);
  std::vector<long> wstart(n);
  std::vector<int> wcount(n, 1);
  std::vector<float> init((size_t)n * S2), e((size_t)n * S2);
  for (int i = 0; i < n; ++i) {  // [2][n][128] -> [n][2][128]
    wstart[i] = i;
    std::memcpy(&init[(size_t)i * S2], state + (size_t)i * VH, VH * 4);
    std::memcpy(&init[(size_t)i * S2 + VH], state + ((size_t)n + i) * VH, VH * 4);
  }
  ZASR_HIP_CHECK(hipMemcpyAsync(d_in, input, (size_t)n * VIN * 4, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_init, init.data(), init.size() * 4, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_ws, wstart.data(), (size_t)n * 8, hipMemcpyHostToDevice, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(d_wc, wcount.data(), (size_t)n * 4, hipMemcpyHostToDevice, st_));
  VadFramesArgs fa{};
  fa.rows576 = d_in;
  fa.frames = ws<float>("frames", (size_t)n * VFR * VFL);
  launch_vad_frames(fa, n, st_);
  float* GX = encode(n);
  VadLstmArgs la{};
  la.gx = GX;
  la.whh = whh_;
  la.bhh = bhh_;
  la.wd = wd_;
  la.bd = bd_;
  la.seg_start = d_ws;
  la.seg_count = d_wc;
  la.init = d_init;
  la.e_out = d_e;
  la.probs = d_p;
  launch_vad_lstm(la, n, st_);
  ZASR_HIP_CHECK(hipMemcpyAsync(prob, d_p, (size_t)n * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipMemcpyAsync(e.data(), d_e, e.size() * 4, hipMemcpyDeviceToHost, st_));
  ZASR_HIP_CHECK(hipStreamSynchronize(st_));
  for (int i = 0; i < n; ++i) {
    std::memcpy(state_out + (size_t)i * VH, &e[(size_t)i * S2], VH * 4);
    std::memcpy(state_out + ((size_t)n + i) * VH, &e[(size_t)i * S2 + VH], VH * 4);
  }
}

}  // namespace zasr
