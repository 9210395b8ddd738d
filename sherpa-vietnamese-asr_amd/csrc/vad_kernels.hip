// Silero VAD (16 kHz, v5 graph) kernels other than the projections, which run on the exact-f32
// MFMA GEMM (gemm.hip: the STFT basis conv, the four encoder convs as im2col GEMMs with the
// ReLU epilogue, the LSTM input projection for every window at once).  SURVEY §8f row 4; the
// loop they replace is core/vad_utils.py:80-111 (one ORT call per 512-sample window).
//
// The recurrence is the only sequential part: one workgroup per stream (file) walks its windows,
// W_hh resident in VGPRs (one gate row per thread), h broadcast from LDS.
#include "common.h"
#include "kernels.h"

namespace zasr {

namespace {
constexpr int VW = 512, VCTX = 64, VFL = 256, VHOP = 128, VFR = 4, VIN = VCTX + VW;

__device__ __forceinline__ float vad_sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// window g of the job -> file index (binary search over the window prefix)
__device__ __forceinline__ int window_file(const long* win_start, int n_files, long g) {
  int lo = 0, hi = n_files - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (win_start[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}
}  // namespace

// per-file max |x| as float bits (non-negative floats order like their bit patterns)
__global__ void vad_maxabs_kernel(const float* __restrict__ audio, const long* __restrict__ off,
                                  const long* __restrict__ len, unsigned* __restrict__ mx) {
  const int f = blockIdx.y;
  const long n = len[f];
  const float* a = audio + off[f];
  float m = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(a[i]));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0 && m > 0.f) atomicMax(mx + f, __float_as_uint(m));
}

// STFT frames of every window: row (g, f) = padded[128 f .. 128 f + 255] where padded =
// [64 context | 512 window | ReflectionPad1d((0, 64))], times the file's boost factor.
// File mode: the context is the previous window's last 64 samples (zeros for window 0).
// Row mode (rows576 != nullptr): window g's 576 input samples are given explicitly.
__global__ __launch_bounds__(256) void vad_frames_kernel(VadFramesArgs a) {
  const long g = blockIdx.x;
  const int t = threadIdx.x;
  const float* src;
  float scale = 1.f;
  bool first = false;
  if (a.rows576) {
    src = a.rows576 + g * VIN;
  } else {
    const int f = window_file(a.win_start, a.n_files, g);
    const long w = g - a.win_start[f];
    src = a.audio + a.off[f] + w * VW - VCTX;  // src[j] = x(j)
    first = (w == 0);
    if (a.maxabs) {
      const float m = __uint_as_float(a.maxabs[f]);
      if (m > 1e-6f && m < 0.071f) scale = 0.071f / m;  // core/vad_utils.py:203-208 (f32)
    }
  }
  float* out = a.frames + g * (VFR * VFL);
#pragma unroll
  for (int fr = 0; fr < VFR; ++fr) {
    int j = fr * VHOP + t;                  // 0 .. 639
    if (j >= VIN) j = 2 * (VIN - 1) - j;    // reflect (edge excluded)
    const float v = (first && j < VCTX) ? 0.f : src[j];
    out[fr * VFL + t] = v * scale;
  }
}

// |STFT| (sqrt(re^2 + im^2), no contraction) laid out as conv1's im2col rows:
// A[(g, t)][k * bins + c] = mag[g][t + k - 1][c]  (0 outside 0..3), K padded with zeros.
__global__ void vad_mag_im2col_kernel(const float* __restrict__ S, int ldS, int bins, int Kp,
                                      float* __restrict__ A) {
  const long row = blockIdx.x;  // (g, t)
  const long g = row / VFR;
  const int t = (int)(row % VFR);
  float* dst = A + row * Kp;
  for (int i = threadIdx.x; i < Kp; i += blockDim.x) {
    float v = 0.f;
    if (i < 3 * bins) {
      const int k = i / bins, c = i - k * bins, tt = t + k - 1;
      if (tt >= 0 && tt < VFR) {
        const float* s = S + (g * VFR + tt) * ldS;
        const float re = s[c], im = s[bins + c];
        v = __fsqrt_rn(__fadd_rn(__fmul_rn(re, re), __fmul_rn(im, im)));
      }
    }
    dst[i] = v;
  }
}

// im2col of a Conv1d(k 3, pad 1, stride s) input held as [N * T][C]:
// A[(n, t')][k * C + c] = Y[n * T + t' * s + k - 1][c] (0 outside 0..T-1)
__global__ void vad_im2col_kernel(const float* __restrict__ Y, int T, int C, int stride, int Tout,
                                  float* __restrict__ A) {
  const long row = blockIdx.x;
  const long n = row / Tout;
  const int to = (int)(row % Tout);
  float* dst = A + row * (3 * C);
  for (int i = threadIdx.x; i < 3 * C; i += blockDim.x) {
    const int k = i / C, c = i - k * C, t = to * stride + k - 1;
    dst[i] = (t >= 0 && t < T) ? Y[(n * T + t) * C + c] : 0.f;
  }
}

// LSTMCell recurrence + decoder head, one segment of one stream per workgroup (512 threads =
// 4 x 128 gate rows, torch order i, f, g, o; every wave holds rows of one gate type, so each
// thread applies its gate's own nonlinearity).  gx[w][512] = x_w W_ih^T + b_ih for every
// window w (GEMM); per step: gates = (gx + h W_hh^T) + b_hh; c = f c + i g; h = o tanh(c);
// prob = sigmoid(relu(h) . wd + bd).
// Segment s covers windows [seg_start - seg_warm, seg_start + seg_count): it starts from
// init[s] = (h, c), runs seg_warm warm-up windows without writing probabilities, stores the
// state reached at seg_start in s_out[s] and the final state in e_out[s] (parallel-in-time
// decode of one long file, verified bit-exactly by the host: VadEngine::probs_device).
__global__ __launch_bounds__(512) void vad_lstm_kernel(VadLstmArgs a) {
  constexpr int H = 128;
  typedef float f2 __attribute__((ext_vector_type(2)));
  __shared__ float4 sh4[H / 4];
  __shared__ float sg[4 * H];
  __shared__ float spart[2][2];
  const int s = blockIdx.x;
  const int j = threadIdx.x;
  const int warm = a.seg_warm ? a.seg_warm[s] : 0;
  const long w0 = a.seg_start[s] - warm;
  const int n = a.seg_count[s] + warm;
  f2 wr[H / 2];
  {
    const float4* r = reinterpret_cast<const float4*>(a.whh + (long)j * H);
#pragma unroll
    for (int q = 0; q < H / 4; ++q) {
      const float4 v = r[q];
      wr[2 * q] = f2{v.x, v.y};
      wr[2 * q + 1] = f2{v.z, v.w};
    }
  }
  const float bj = a.bhh[j];
  const int gate = j >> 7;  // 0 i, 1 f, 2 g, 3 o (uniform per wave)
  float c = 0.f, wdk = 0.f;
  float* sh = reinterpret_cast<float*>(sh4);
  if (j < H) {
    wdk = a.wd[j];
    sh[j] = a.init ? a.init[(long)s * 2 * H + j] : 0.f;
    c = a.init ? a.init[(long)s * 2 * H + H + j] : 0.f;
  }
  __syncthreads();
  float gnext = n > 0 ? a.gx[w0 * (4 * H) + j] : 0.f;
  for (int t = 0; t < n; ++t) {
    if (t == warm && a.s_out && j < H) {  // state at the segment start
      a.s_out[(long)s * 2 * H + j] = sh[j];
      a.s_out[(long)s * 2 * H + H + j] = c;
    }
    const float gcur = gnext;
    if (t + 1 < n) gnext = a.gx[(w0 + t + 1) * (4 * H) + j];
    f2 acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < H / 4; ++q) {
      const float4 hv = sh4[q];
      acc0 = __builtin_elementwise_fma(wr[2 * q], f2{hv.x, hv.y}, acc0);
      acc1 = __builtin_elementwise_fma(wr[2 * q + 1], f2{hv.z, hv.w}, acc1);
    }
    const float pre = (gcur + ((acc0.x + acc0.y) + (acc1.x + acc1.y))) + bj;
    sg[j] = gate == 2 ? tanhf(pre) : vad_sigmoid(pre);
    __syncthreads();
    if (j < H) {
      c = sg[H + j] * c + sg[j] * sg[2 * H + j];
      const float h = sg[3 * H + j] * tanhf(c);
      sh[j] = h;
      float v = fmaxf(h, 0.f) * wdk;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((j & 63) == 0) spart[t & 1][j >> 6] = v;
    }
    __syncthreads();
    if (j == 0 && t >= warm)
      a.probs[w0 + t] = vad_sigmoid((spart[t & 1][0] + spart[t & 1][1]) + a.bd);
  }
  if (j < H) {
    if (n == warm && a.s_out) {
      a.s_out[(long)s * 2 * H + j] = sh[j];
      a.s_out[(long)s * 2 * H + H + j] = c;
    }
    if (a.e_out) {
      a.e_out[(long)s * 2 * H + j] = sh[j];
      a.e_out[(long)s * 2 * H + H + j] = c;
    }
  }
}

void launch_vad_maxabs(const float* audio, const long* off, const long* len, int n_files,
                       unsigned* mx, hipStream_t st) {
  if (n_files <= 0) return;
  ZASR_LAUNCH(vad_maxabs_kernel, dim3(64, n_files), dim3(256), 0, st, audio, off, len, mx);
}

void launch_vad_frames(const VadFramesArgs& a, long n_windows, hipStream_t st) {
  if (n_windows <= 0) return;
  ZASR_LAUNCH(vad_frames_kernel, dim3((unsigned)n_windows), dim3(256), 0, st, a);
}

void launch_vad_mag_im2col(const float* S, int ldS, int bins, int Kp, long n_windows, float* A,
                           hipStream_t st) {
  if (n_windows <= 0) return;
  ZASR_LAUNCH(vad_mag_im2col_kernel, dim3((unsigned)(n_windows * VFR)), dim3(128), 0, st, S,
                     ldS, bins, Kp, A);
}

void launch_vad_im2col(const float* Y, long N, int T, int C, int stride, int Tout, float* A,
                       hipStream_t st) {
  if (N <= 0) return;
  ZASR_LAUNCH(vad_im2col_kernel, dim3((unsigned)(N * Tout)), dim3(128), 0, st, Y, T, C,
                     stride, Tout, A);
}

void launch_vad_lstm(const VadLstmArgs& a, int n_segments, hipStream_t st) {
  if (n_segments <= 0) return;
  ZASR_LAUNCH(vad_lstm_kernel, dim3(n_segments), dim3(512), 0, st, a);
}

}  // namespace zasr
