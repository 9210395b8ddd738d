// Non-GEMM kernels of the encoder path: fbank, Conv2dSubsampling convs, attention softmax,
// and the Zipformer2 elementwise / per-sequence operators.  All HBM-streaming kernels read
// and write row-contiguous activations with float4 per lane where the width allows.
#include "common.h"
#include "kernels.h"

namespace zasr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// index of the sequence that owns packed row `r`: largest b with off[b] <= r
__device__ __forceinline__ int find_seq(const int* off, int nseq, int r) {
  int lo = 0, hi = nseq - 1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= r) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// row -> sequence map of one time resolution (built once per batch)
__global__ void row2seq_kernel(const int* __restrict__ off, int nseq, int total,
                               int* __restrict__ map) {
  int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < total) map[r] = find_seq(off, nseq, r);
}

void launch_row2seq(const int* off, int nseq, int total, int* map, hipStream_t st) {
  if (total <= 0) return;
  ZASR_LAUNCH(row2seq_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, off, nseq, total,
                     map);
}

// =====================================================================================
// fbank: one wave per frame, 4 frames per block.  Samples gathered with kaldi edge
// reflection (one round trip: all 7 loads per lane in flight), DC removal, pre-emphasis
// (left neighbour by lane shuffle) and povey window in f32; the 512-point real FFT in f64
// (knf's rdft runs in double) as a 256-point complex FFT of z[n] = x[2n] + i x[2n+1]:
// four radix-4 Stockham passes, one butterfly per lane per pass, ping-ponging two per-wave
// LDS images (no bit reversal, wave-local barriers only), then the even/odd split
// X[k] = E[k] + W512^k O[k]; power spectrum f32, mel triangles (tables in LDS), log with
// FLT_EPSILON floor.
// CAMPP = true: the CAM++ front end instead (core/speaker_diarization_senko_campp_optimized.py:
// 86-159): samples x 32768, snip_edges framing (frame f = samples 160 f .. 160 f + 399), the
// first sample's pre-emphasis uses the previous SIGNAL sample (0 for frame 0), mel bank
// 20 Hz .. Nyquist, floor 1.0 (CMVN follows in campp_cmvn_kernel).
// =====================================================================================
constexpr int kFbWaves = 4;
constexpr int kMelWMax = 512;   // each FFT bin lies in at most two triangles
constexpr int kFbSeqLds = 1024; // sequence offsets staged in LDS up to this many sequences
constexpr int kFbBlocks = 2048; // grid-stride: 8 blocks per CU, each wave ~50 frames per hour

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

template <bool CAMPP>
__global__ __launch_bounds__(64 * kFbWaves) void fbank_kernel(
    const float* __restrict__ wav, const long* __restrict__ wav_off,
    const int* __restrict__ nsamp, const int* __restrict__ fr_off, int nseq, int total_frames,
    FbankTables tabs, float* __restrict__ out) {
  __shared__ double2 sTw[256];  // exp(-2 pi i u / 512), u < 256
  __shared__ float sWin[400];
  __shared__ int sMeta[240];
  __shared__ float sMelW[kMelWMax];
  __shared__ double2 sA[kFbWaves][256], sB[kFbWaves][256];
  __shared__ int sOff[kFbSeqLds + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // sequence frame offsets in LDS when they fit (the per-frame sequence search then costs
  // LDS round trips, not L2 ones)
  const bool off_lds = nseq <= kFbSeqLds;
  if (off_lds)
    for (int i = tid; i <= nseq; i += 64 * kFbWaves) sOff[i] = fr_off[i];
  for (int i = tid; i < 256; i += 64 * kFbWaves)
    sTw[i] = make_double2(tabs.twiddle[2 * i], tabs.twiddle[2 * i + 1]);
  for (int i = tid; i < 400; i += 64 * kFbWaves) sWin[i] = tabs.window[i];
  if (tid < 80) {
    sMeta[tid] = tabs.mel_start[tid];
    sMeta[80 + tid] = tabs.mel_len[tid];
    sMeta[160 + tid] = tabs.mel_woff[tid];
  }
  {
    const int nw = tabs.mel_woff[79] + tabs.mel_len[79];
    for (int i = tid; i < nw && i < kMelWMax; i += 64 * kFbWaves) sMelW[i] = tabs.mel_w[i];
  }
  __syncthreads();  // tables staged
  const int* offs = off_lds ? sOff : fr_off;
  // grid-stride over frames: each wave takes frames w + kFbWaves * blockIdx.x + k * stride, so
  // the tables are staged once per block, not once per 4 frames.  The samples of the wave's
  // NEXT frame are gathered before the current frame is computed (7 loads per lane in flight
  // under the FFT and mel work; the index is clamped, so the loads are unconditional and the
  // waits stay counted)
  const int stride = gridDim.x * kFbWaves;
  auto gather = [&](int frame, float (&x)[7], float& ctx, int& f) {
    const int b = find_seq(offs, nseq, frame);
    f = frame - offs[b];
    const long n = nsamp[b];
    const float* base = wav + wav_off[b];
    if constexpr (CAMPP) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int i = lane + 64 * k;
        x[k] = base[(long)f * 160 + (i < 400 ? i : 399)];
      }
      ctx = base[f > 0 ? (long)f * 160 - 1 : 0];
    } else {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const int i = lane + 64 * k;
        long s = (long)f * 160 - 120 + (i < 400 ? i : 399);
        while (s < 0 || s >= n) s = (s < 0) ? (-s - 1) : (2L * n - 1 - s);
        x[k] = base[s];
      }
      ctx = 0.f;
    }
  };
  const int first = blockIdx.x * kFbWaves + w;
  float xn[7], ctxn = 0.f;
  int fn = 0;
  if (first < total_frames) gather(first, xn, ctxn, fn);
  for (int frame = first; frame < total_frames; frame += stride) {
  float xv[7];
  float ctx0 = 0.f;  // CAMPP: the signal sample before the frame (scaled; 0 for frame 0)
  {
#pragma unroll
    for (int k = 0; k < 7; ++k) xv[k] = xn[k];
    const int f0 = fn;
    if constexpr (CAMPP) {
#pragma unroll
      for (int k = 0; k < 7; ++k) xv[k] *= 32768.0f;
      ctx0 = f0 > 0 ? ctxn * 32768.0f : 0.f;
    }
    const int nxt = frame + stride < total_frames ? frame + stride : total_frames - 1;
    gather(nxt, xn, ctxn, fn);
    double part = 0.0;
#pragma unroll
    for (int k = 0; k < 7; ++k)
      if (lane + 64 * k < 400) part += (double)xv[k];
    const float mean = (float)(wave_sum_d(part) / 400.0);
#pragma unroll
    for (int k = 0; k < 7; ++k) xv[k] = xv[k] - mean;
  }
  double2* A = sA[w];
  double2* B = sB[w];
  {
    // pre-emphasis (left neighbour of sample i = lane + 64k: lane - 1, or lane 63 of chunk
    // k - 1; sample 0 uses itself), window; real samples into A viewed as double[512]
    double* xr = reinterpret_cast<double*>(A);
    float carry = 0.f;
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      const float up = __shfl(xv[k], lane == 0 ? 0 : lane - 1, 64);
      const float prev = lane != 0 ? up : (k == 0 ? (CAMPP ? ctx0 : xv[0]) : carry);
      carry = __shfl(xv[k], 63, 64);
      const int i = lane + 64 * k;
      const float e = __fsub_rn(xv[k], __fmul_rn(0.97f, prev));
      xr[i] = i < 400 ? (double)__fmul_rn(e, sWin[i < 400 ? i : 0]) : 0.0;
    }
    xr[lane + 448] = 0.0;
  }
  __builtin_amdgcn_wave_barrier();
  // 256-point complex FFT (Stockham radix-4): pass s with Ns = 4^s, lane j = one butterfly
  const int j = lane;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const double2* X = (s & 1) ? B : A;
    double2* Y = (s & 1) ? A : B;
    const int ns_log = 2 * s, Ns = 1 << ns_log;
    const int k = j & (Ns - 1);
    double2 v0 = X[j], v1 = X[j + 64], v2 = X[j + 128], v3 = X[j + 192];
    if (s > 0) {
      // twiddle exp(-2 pi i k r / (4 Ns)) = W512^(u r), u = k * 128 / Ns
      const int u = k << (7 - ns_log);
      const int u2 = 2 * u, u3 = 3 * u;
      const double2 t1 = sTw[u];
      const double2 t2 = u2 < 256 ? sTw[u2] : make_double2(-sTw[u2 - 256].x, -sTw[u2 - 256].y);
      const double2 t3 = u3 < 256 ? sTw[u3] : make_double2(-sTw[u3 - 256].x, -sTw[u3 - 256].y);
      v1 = cmul(v1, t1);
      v2 = cmul(v2, t2);
      v3 = cmul(v3, t3);
    }
    const double2 a0 = make_double2(v0.x + v2.x, v0.y + v2.y);
    const double2 a1 = make_double2(v0.x - v2.x, v0.y - v2.y);
    const double2 a2 = make_double2(v1.x + v3.x, v1.y + v3.y);
    const double2 a3 = make_double2(v1.y - v3.y, v3.x - v1.x);  // (v1 - v3) * (-i)
    const int o = ((j >> ns_log) << (ns_log + 2)) + k;
    Y[o] = make_double2(a0.x + a2.x, a0.y + a2.y);
    Y[o + Ns] = make_double2(a1.x + a3.x, a1.y + a3.y);
    Y[o + 2 * Ns] = make_double2(a0.x - a2.x, a0.y - a2.y);
    Y[o + 3 * Ns] = make_double2(a1.x - a3.x, a1.y - a3.y);
    __builtin_amdgcn_wave_barrier();
  }
  // Z = FFT256(z) is in A; X[k] = E[k] + W512^k O[k], E = (Z_k + conj Z_-k) / 2,
  // O = (Z_k - conj Z_-k) / 2i; power of bins 0..255 (f32) into B viewed as float[256]
  float* pw = reinterpret_cast<float*>(B);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int kb = lane + 64 * q;
    const double2 zk = A[kb], zm = A[(256 - kb) & 255];
    const double2 E = make_double2(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
    const double2 O = make_double2(0.5 * (zk.y + zm.y), -0.5 * (zk.x - zm.x));
    const double2 X = cmul(O, sTw[kb]);
    const float re = (float)(E.x + X.x), im = (float)(E.y + X.y);
    pw[kb] = __fadd_rn(__fmul_rn(re, re), __fmul_rn(im, im));
  }
  __builtin_amdgcn_wave_barrier();
  for (int m = lane; m < 80; m += 64) {
    const int st = sMeta[m], ln = sMeta[80 + m], wo = sMeta[160 + m];
    // the taps in order (the same fma chain), four LDS pairs read ahead of their fmas
    float acc = 0.f;
    int k = 0;
    for (; k + 4 <= ln; k += 4) {
      const float w0 = sMelW[wo + k], w1 = sMelW[wo + k + 1], w2 = sMelW[wo + k + 2], w3 = sMelW[wo + k + 3];
      const float p0 = pw[st + k], p1 = pw[st + k + 1], p2 = pw[st + k + 2], p3 = pw[st + k + 3];
      acc = fmaf(w0, p0, acc);
      acc = fmaf(w1, p1, acc);
      acc = fmaf(w2, p2, acc);
      acc = fmaf(w3, p3, acc);
    }
    for (; k < ln; ++k) acc = fmaf(sMelW[wo + k], pw[st + k], acc);
    out[(long)frame * 80 + m] = logf(fmaxf(acc, CAMPP ? 1.0f : 1.1920928955078125e-07f));
  }
  __builtin_amdgcn_wave_barrier();  // the next frame rewrites this wave's A / B images
  }
}

void launch_fbank(const float* wav, const long* wav_off, const int* nsamp, const int* fr_off,
                  int nseq, int total_frames, const FbankTables& tabs, float* out,
                  hipStream_t st, bool campp) {
  if (total_frames <= 0) return;
  if (campp)
    ZASR_LAUNCH(fbank_kernel<true>, dim3(std::min(cdiv(total_frames, kFbWaves), kFbBlocks)),
                       dim3(64 * kFbWaves), 0, st, wav, wav_off, nsamp, fr_off, nseq, total_frames,
                       tabs, out);
  else
    ZASR_LAUNCH(fbank_kernel<false>, dim3(std::min(cdiv(total_frames, kFbWaves), kFbBlocks)),
                       dim3(64 * kFbWaves), 0, st, wav, wav_off, nsamp, fr_off, nseq, total_frames,
                       tabs, out);
}

// =====================================================================================
// The planner's silence detector (core/asr_engine.py:521-554 find_silent_regions):
//   energies = sqrt(mean(frames ** 2, axis=1)) < threshold
// in numpy's float32 arithmetic, bit for bit.  numpy reduces each row with its pairwise sum
// (numpy/_core/src/umath/loops_utils.h.src pairwise_sum): n <= 128 -> eight running partial
// sums over blocks of 8, combined as ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the tail in
// order; n > 128 -> the halves [0, n2) and [n2, n) with n2 = n/2 rounded down to a multiple
// of 8, summed separately and added.  Then / n (f32 true divide), sqrt (correctly rounded),
// and the comparison in f32 (a Python float threshold is cast to the array's f32).  No
// square and add may contract into an FMA (see np_pairwise_sq).
// One thread per frame; the frame's row is read as float4s (rows are 16-byte aligned when
// frame_len % 4 == 0, host-checked).  HBM-bound: 4 B per sample.
// =====================================================================================
// HIP's __fadd_rn / __fmul_rn are plain operators (contractible into FMAs) and __fsqrt_rn is
// the native sqrt unless OCML_BASIC_ROUNDED_OPERATIONS is set (clang __clang_hip_math.h): the
// code below turns contraction off and uses sqrtf / '/', which hipcc lowers correctly rounded
// (-fhip-fp32-correctly-rounded-divide-sqrt is the default).
__device__ __forceinline__ float np_pairwise_sq(const float* x, int n) {
#pragma clang fp contract(off)
  // n <= 128: numpy's unrolled block sum of x[i]^2
  if (n < 8) {
    float s = -0.0f;
    for (int i = 0; i < n; ++i) s = s + x[i] * x[i];
    return s;
  }
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = x[j] * x[j];
  int i = 8;
  const int nb = n - (n % 8);
  for (; i < nb; i += 8) {
    const float4 a = *reinterpret_cast<const float4*>(x + i);
    const float4 b = *reinterpret_cast<const float4*>(x + i + 4);
    r[0] = r[0] + a.x * a.x;
    r[1] = r[1] + a.y * a.y;
    r[2] = r[2] + a.z * a.z;
    r[3] = r[3] + a.w * a.w;
    r[4] = r[4] + b.x * b.x;
    r[5] = r[5] + b.y * b.y;
    r[6] = r[6] + b.z * b.z;
    r[7] = r[7] + b.w * b.w;
  }
  float s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) s = s + x[i] * x[i];
  return s;
}

__global__ __launch_bounds__(256) void silence_flags_kernel(const float* __restrict__ wav,
                                                            long nframes, int flen, int n2,
                                                            float threshold,
                                                            unsigned char* __restrict__ flags) {
#pragma clang fp contract(off)
  const long f = (long)blockIdx.x * 256 + threadIdx.x;
  if (f >= nframes) return;
  const float* x = wav + f * flen;
  float s;
  if (n2 == 0) {
    s = np_pairwise_sq(x, flen);
  } else {
    s = np_pairwise_sq(x, n2) + np_pairwise_sq(x + n2, flen - n2);
  }
  const float e = sqrtf(s / (float)flen);
  flags[f] = e < threshold ? 1 : 0;
}

__global__ void selftest_noop_kernel(int* sink) {
  if (sink && threadIdx.x == 0xffffff) *sink = 0;
}

void launch_selftest_noop(int block_threads) {
  ZASR_LAUNCH(selftest_noop_kernel, dim3(1), dim3(block_threads), 0, nullptr, nullptr);
  ZASR_HIP_CHECK(hipDeviceSynchronize());
}

void launch_silence_flags(const float* wav, long n, int frame_len, float threshold,
                          unsigned char* flags, hipStream_t st) {
  ZASR_REQUIRE(frame_len > 0 && frame_len % 4 == 0,
               "silence flags: frame length must be a positive multiple of 4 samples");
  ZASR_REQUIRE((reinterpret_cast<uintptr_t>(wav) & 15) == 0,
               "silence flags: the signal must be 16-byte aligned");
  // numpy's split (n > 128): halves of n2 = (n / 2) rounded down to 8 and n - n2, each <= 128
  int n2 = 0;
  if (frame_len > 128) {
    n2 = frame_len / 2;
    n2 -= n2 % 8;
    ZASR_REQUIRE(n2 <= 128 && frame_len - n2 <= 128,
                 "silence flags: frame length above 256 samples (numpy's deeper split) unsupported");
  }
  const long nframes = n / frame_len;
  if (nframes <= 0) return;
  ZASR_LAUNCH(silence_flags_kernel, dim3((unsigned)cdivl(nframes, 256)), dim3(256), 0, st,
                     wav, nframes, frame_len, n2, threshold, flags);
}

// =====================================================================================
// conv.0: Conv2d(1 -> 8, 3x3, padding (0, 1)) + SwooshR.  One thread per (t, f).
// =====================================================================================
// BF16: bf16 output and the native-exp/log SwooshR (the bf16 mode; conv.4 reads it through
// its bf16 implicit-im2col loader); f32: the libm form (fp32, bf16x3, bf16x6), or with FAST the
// native form (f16x3, whose GEMM epilogues' SwooshR is swooshr_fast too; in bf16x6 the native
// form flipped a near-tie beam chunk of the widened oracle set, so that mode keeps libm)
template <bool BF16, bool FAST = BF16>
__global__ void conv1_kernel(const float* __restrict__ fb, const int* __restrict__ fb_off,
                             const int* __restrict__ c1_off, const int* __restrict__ c1_map,
                             int total,
                             const float* __restrict__ w, const float* __restrict__ bias,
                             void* __restrict__ out) {
  int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total * 80) return;
  int row = e / 80, f = e - row * 80;
  int b = c1_map[row];
  int t = row - c1_off[b];
  const float* src = fb + (long)(fb_off[b] + t) * 80;
  float xin[9];
#pragma unroll
  for (int kt = 0; kt < 3; ++kt)
#pragma unroll
    for (int kf = 0; kf < 3; ++kf) {
      const int ff = f + kf - 1;
      const float v = src[kt * 80 + (ff < 0 ? 0 : (ff > 79 ? 79 : ff))];  // unconditional
      xin[kt * 3 + kf] = (ff >= 0 && ff < 80) ? v : 0.f;
    }
  float r[8];
#pragma unroll
  for (int o = 0; o < 8; ++o) {
    float acc = bias[o];
#pragma unroll
    for (int k = 0; k < 9; ++k) acc = fmaf(w[o * 9 + k], xin[k], acc);
    r[o] = FAST ? swooshr_fast(acc) : swooshr(acc);
  }
  if constexpr (BF16) {
    typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
    bf16x8_t h;
#pragma unroll
    for (int o = 0; o < 8; ++o) h[o] = (__bf16)r[o];
    reinterpret_cast<bf16x8_t*>(out)[e] = h;
  } else {
    float4* dst = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + (long)e * 8);
    dst[0] = make_float4(r[0], r[1], r[2], r[3]);
    dst[1] = make_float4(r[4], r[5], r[6], r[7]);
  }
}

void launch_conv1(const float* fb, const int* fb_off, const int* c1_off, const int* c1_map,
                  int total_rows, const float* w, const float* b, void* out, bool out_bf16,
                  hipStream_t st, bool fast) {
  if (total_rows <= 0) return;
  long n = (long)total_rows * 80;
  if (out_bf16)
    ZASR_LAUNCH(conv1_kernel<true>, dim3(cdivl(n, 256)), dim3(256), 0, st, fb, fb_off,
                       c1_off, c1_map, total_rows, w, b, out);
  else if (fast)
    ZASR_LAUNCH((conv1_kernel<false, true>), dim3(cdivl(n, 256)), dim3(256), 0, st, fb,
                       fb_off, c1_off, c1_map, total_rows, w, b, out);
  else
    ZASR_LAUNCH(conv1_kernel<false>, dim3(cdivl(n, 256)), dim3(256), 0, st, fb, fb_off,
                       c1_off, c1_map, total_rows, w, b, out);
}


// =====================================================================================
// BiasNorm (+ optional bypass): one wave per row.
// =====================================================================================
template <int NQ>  // float4 per lane: d <= 256 * NQ
__global__ __launch_bounds__(256) void bias_norm_kernel(float* __restrict__ x, int rows, int d,
                                                        const float* __restrict__ bias, float scale,
                                                        const float* __restrict__ orig,
                                                        const float* __restrict__ bscale,
                                                        float* __restrict__ copy_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int d4 = d >> 2;
  float4* xr = reinterpret_cast<float4*>(x + (long)row * d);
  float4 v[NQ], o[NQ];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = lane + 64 * q;
    const int ic = i < d4 ? i : d4 - 1;
    v[q] = xr[ic];
    if (orig) o[q] = reinterpret_cast<const float4*>(orig + (long)row * d)[ic];
    const float4 bq = reinterpret_cast<const float4*>(bias)[ic];
    float4 t = make_float4(v[q].x - bq.x, v[q].y - bq.y, v[q].z - bq.z, v[q].w - bq.w);
    if (i >= d4) t = make_float4(0.f, 0.f, 0.f, 0.f);
    ss = fmaf(t.x, t.x, fmaf(t.y, t.y, fmaf(t.z, t.z, fmaf(t.w, t.w, ss))));
  }
  ss = wave_sum(ss);
  const float k = scale / sqrtf(ss / (float)d);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int i = lane + 64 * q;
    if (i >= d4) continue;
    float4 r = make_float4(v[q].x * k, v[q].y * k, v[q].z * k, v[q].w * k);
    if (orig) {
      const float4 s4 = reinterpret_cast<const float4*>(bscale)[i];
      r = make_float4(o[q].x + (r.x - o[q].x) * s4.x, o[q].y + (r.y - o[q].y) * s4.y,
                      o[q].z + (r.z - o[q].z) * s4.z, o[q].w + (r.w - o[q].w) * s4.w);
    }
    xr[i] = r;
    // the next layer's bypass input (its copy of src): the row is complete in this thread's
    // registers, so writing it over `orig` (read above by the same lane) is safe
    if (copy_out) reinterpret_cast<float4*>(copy_out + (long)row * d)[i] = r;
  }
}

void launch_bias_norm(float* x, int rows, int d, const float* bias, float log_scale,
                      const float* orig, const float* bypass_scale, hipStream_t st,
                      float* copy_out) {
  if (rows <= 0) return;
  ZASR_REQUIRE(d % 4 == 0 && d <= 1024, "BiasNorm width must be a multiple of 4, <= 1024");
  const dim3 grid(cdiv(rows, 4));
  if (d <= 256)
    ZASR_LAUNCH(bias_norm_kernel<1>, grid, dim3(256), 0, st, x, rows, d, bias,
                       expf(log_scale), orig, bypass_scale, copy_out);
  else if (d <= 512)
    ZASR_LAUNCH(bias_norm_kernel<2>, grid, dim3(256), 0, st, x, rows, d, bias,
                       expf(log_scale), orig, bypass_scale, copy_out);
  else
    ZASR_LAUNCH(bias_norm_kernel<4>, grid, dim3(256), 0, st, x, rows, d, bias,
                       expf(log_scale), orig, bypass_scale, copy_out);
}

// =====================================================================================
// elementwise: bypass, GLU, nonlin prep (float4 over channels; d % 4 == 0)
// =====================================================================================
__global__ void bypass_kernel(float* __restrict__ x, const float* __restrict__ orig,
                              const float* __restrict__ s, long n4, int d4) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  int c4 = (int)(i % d4);
  float4 v = reinterpret_cast<float4*>(x)[i];
  float4 o = reinterpret_cast<const float4*>(orig)[i];
  float4 k = reinterpret_cast<const float4*>(s)[c4];
  v.x = o.x + (v.x - o.x) * k.x;
  v.y = o.y + (v.y - o.y) * k.y;
  v.z = o.z + (v.z - o.z) * k.z;
  v.w = o.w + (v.w - o.w) * k.w;
  reinterpret_cast<float4*>(x)[i] = v;
}

void launch_bypass(float* x, const float* orig, const float* s, long rows, int d,
                   hipStream_t st) {
  long n4 = rows * d / 4;
  if (n4 <= 0) return;
  ZASR_LAUNCH(bypass_kernel, dim3(cdivl(n4, 256)), dim3(256), 0, st, x, orig, s, n4,
                     d / 4);
}

__global__ void glu_kernel(const float* __restrict__ x2, float* __restrict__ g, long n4,
                           int d4) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  long r = i / d4;
  int c4 = (int)(i - r * d4);
  const float4* row = reinterpret_cast<const float4*>(x2) + r * 2 * d4;
  float4 a = row[c4], s = row[d4 + c4];
  float4 o;
  o.x = a.x * sigmoidf_(s.x);
  o.y = a.y * sigmoidf_(s.y);
  o.z = a.z * sigmoidf_(s.z);
  o.w = a.w * sigmoidf_(s.w);
  reinterpret_cast<float4*>(g)[i] = o;
}

void launch_glu(const float* x2, float* g, long rows, int d, hipStream_t st) {
  long n4 = rows * d / 4;
  if (n4 <= 0) return;
  ZASR_LAUNCH(glu_kernel, dim3(cdivl(n4, 256)), dim3(256), 0, st, x2, g, n4, d / 4);
}

__global__ void nonlin_prep_kernel(const float* __restrict__ h3, float* __restrict__ t1, long n4,
                                   int h4) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  long r = i / h4;
  int c4 = (int)(i - r * h4);
  const float4* row = reinterpret_cast<const float4*>(h3) + r * 3 * h4;
  float4 s = row[c4], x = row[h4 + c4];
  float4 o;
  o.x = tanhf(s.x) * x.x;
  o.y = tanhf(s.y) * x.y;
  o.z = tanhf(s.z) * x.z;
  o.w = tanhf(s.w) * x.w;
  reinterpret_cast<float4*>(t1)[i] = o;
}

void launch_nonlin_prep(const float* h3, float* t1, long rows, int hid, hipStream_t st) {
  long n4 = rows * hid / 4;
  if (n4 <= 0) return;
  ZASR_LAUNCH(nonlin_prep_kernel, dim3(cdivl(n4, 256)), dim3(256), 0, st, h3, t1, n4,
                     hid / 4);
}

// =====================================================================================
// ConvolutionModule core: GLU (x * sigmoid(s) of the in_proj halves) -> depthwise conv1d
// over time (zero padding per sequence) + bias -> SwooshR.  Block tile: 64 packed rows x
// 64 channels with a K/2 halo staged in LDS as GLU outputs (loads unconditional and batched:
// one memory round trip).  Each lane owns one channel and 16 consecutive rows, so every
// staged value is read from LDS once per lane and feeds up to K FMAs from registers.
// Rows whose window crosses a sequence edge take the masked path (per-row tap range).
// =====================================================================================
constexpr int kDw1T = 64;

// K = compiled window (7, 15, 31); a smaller odd kernel Kr runs with zero taps padded
// symmetrically (adds exact zeros only)
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 ld4(const __bf16* p) {
  const bf16x4_t v = *reinterpret_cast<const bf16x4_t*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}
__device__ __forceinline__ void st1(float* p, float v) { *p = v; }
__device__ __forceinline__ void st1(__bf16* p, float v) { *p = (__bf16)v; }

// GLU = false: x2 is already the GLU output, [rows][d] (split modes: the in_proj GEMM's
// EPI_GLU epilogue applied it, with the same sigmoid_fast)
template <int K, typename TI, typename TO, bool GLU = true>
__global__ __launch_bounds__(256) void glu_dwconv1d_kernel(
    const TI* __restrict__ x2, const int* __restrict__ off, const int* __restrict__ map,
    int total_rows, int d, int Kr, const float* __restrict__ w, const float* __restrict__ bias,
    TO* __restrict__ out) {
  constexpr int half = K / 2;
  constexpr int nrows = kDw1T + K - 1;
  constexpr int nf4 = nrows * 16;
  constexpr int kIt = (nf4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float tile[nrows * 64];
  __shared__ float sW[64 * K];
  __shared__ int sLo[kDw1T], sHi[kDw1T], sMasked;
  const int r0 = blockIdx.x * kDw1T;
  const int c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  if (tid == 0) sMasked = 0;
  // every global load of the block is issued before the first wait: the block's channel
  // weights (staged through LDS: w is [d][Kr], so per-lane loads of a lane's own row would
  // touch one cache line per lane and instruction), the bias, the sequence bounds of the tile
  // rows (map -> off) and the staged input -- one memory round trip
  const int c = tid & 63;
  const int cw = c0 + c < d ? c0 + c : d - 1;  // clamped: lanes past d never store
  const int nw = (d - c0 < 64 ? d - c0 : 64) * Kr;
  constexpr int kWIt = (64 * K + 255) / 256;
  float wl[kWIt];
#pragma unroll
  for (int q = 0; q < kWIt; ++q) {
    const int i = tid + 256 * q;
    wl[q] = w[(long)c0 * Kr + (i < nw ? i : nw - 1)];
  }
  const float bc = bias[cw];
  int seq_lo = 0, seq_hi = 0;
  const int rb = r0 + (tid & (kDw1T - 1));
  if (tid < kDw1T && rb < total_rows) {
    const int b = map[rb];
    seq_lo = off[b];
    seq_hi = off[b + 1];
  }
  {
    float4 a[kIt], g[kIt];
#pragma unroll
    for (int q = 0; q < kIt; ++q) {
      const int e = tid + 256 * q;
      const int c4 = e & 15, rr = e >> 4;
      int r = r0 - half + rr;
      r = r < 0 ? 0 : (r >= total_rows ? total_rows - 1 : r);
      const int cc = c0 + 4 * c4 < d ? c0 + 4 * c4 : d - 4;
      if constexpr (GLU) {
        a[q] = ld4(x2 + (long)r * 2 * d + cc);
        g[q] = ld4(x2 + (long)r * 2 * d + d + cc);
      } else {
        a[q] = ld4(x2 + (long)r * d + cc);
      }
    }
#pragma unroll
    for (int q = 0; q < kIt; ++q) {
      const int e = tid + 256 * q;
      const int c4 = e & 15, rr = e >> 4;
      const int r = r0 - half + rr;
      const bool ok = e < nf4 && r >= 0 && r < total_rows && c0 + 4 * c4 < d;
      float4 v = a[q];
      if constexpr (GLU)
        v = make_float4(a[q].x * sigmoid_fast(g[q].x), a[q].y * sigmoid_fast(g[q].y),
                        a[q].z * sigmoid_fast(g[q].z), a[q].w * sigmoid_fast(g[q].w));
      if (!ok) v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (e < nf4) *reinterpret_cast<float4*>(&tile[rr * 64 + 4 * c4]) = v;
    }
  }
#pragma unroll
  for (int q = 0; q < kWIt; ++q) {
    const int i = tid + 256 * q;
    if (i < nw) sW[i] = wl[q];
  }
  __syncthreads();
  // this lane's taps (zero past Kr, centred): row c of the staged [64][Kr] block, an odd
  // stride, so the 64 lanes' reads fall in distinct banks
  float wr[K];
  {
    const int pad = (K - Kr) / 2;
    const int cl = c0 + c < d ? c : (d - c0) - 1;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int kk = k - pad;
      const bool ok = kk >= 0 && kk < Kr;
      const float wv = sW[cl * Kr + (ok ? kk : 0)];
      wr[k] = ok ? wv : 0.f;
    }
  }
  if (tid < kDw1T) {
    const int r = r0 + tid;
    int lo = -half, hi = half;
    if (r < total_rows) {
      lo = max(seq_lo - r, -half);
      hi = min(seq_hi - 1 - r, half);
    }
    sLo[tid] = lo;
    sHi[tid] = hi;
    if (lo != -half || hi != half) atomicOr(&sMasked, 1);
  }
  __syncthreads();
  if (c0 + c >= d) return;
  const int tr0 = (tid >> 6) * 16;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = bc;
  if (!sMasked) {
#pragma unroll
    for (int rr = 0; rr < 16 + K - 1; ++rr) {
      const float v = tile[(tr0 + rr) * 64 + c];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = rr - i;
        if (k >= 0 && k < K) acc[i] = fmaf(wr[k], v, acc[i]);
      }
    }
  } else {
    int lo[16], hi[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      lo[i] = sLo[tr0 + i];
      hi[i] = sHi[tr0 + i];
    }
#pragma unroll
    for (int rr = 0; rr < 16 + K - 1; ++rr) {
      const float v = tile[(tr0 + rr) * 64 + c];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int k = rr - i;
        if (k >= 0 && k < K && k - half >= lo[i] && k - half <= hi[i]) acc[i] = fmaf(wr[k], v, acc[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + tr0 + i;
    if (r < total_rows) st1(out + (long)r * d + c0 + c, swooshr_fast(acc[i]));
  }
}

template <typename TI, typename TO, bool GLU = true>
static void launch_glu_dwconv1d_t(const TI* x2, const int* off, const int* map, int total_rows,
                                  int d, int K, const float* w, const float* b, TO* out,
                                  hipStream_t st) {
  if (total_rows <= 0) return;
  ZASR_REQUIRE(d % 4 == 0, "conv module channels must be a multiple of 4");
  dim3 grid(cdiv(total_rows, kDw1T), cdiv(d, 64));
  ZASR_REQUIRE(K >= 1 && K <= 31 && (K & 1), "depthwise kernel size must be odd and <= 31");
  if (K <= 7)
    ZASR_LAUNCH((glu_dwconv1d_kernel<7, TI, TO, GLU>), grid, dim3(256), 0, st, x2, off, map, total_rows, d, K, w, b, out);
  else if (K <= 15)
    ZASR_LAUNCH((glu_dwconv1d_kernel<15, TI, TO, GLU>), grid, dim3(256), 0, st, x2, off, map, total_rows, d, K, w, b, out);
  else
    ZASR_LAUNCH((glu_dwconv1d_kernel<31, TI, TO, GLU>), grid, dim3(256), 0, st, x2, off, map, total_rows, d, K, w, b, out);
}

void launch_dwconv1d_post_glu(const float* g, const int* off, const int* map, int total_rows,
                              int d, int K, const float* w, const float* b, float* out,
                              hipStream_t st) {
  launch_glu_dwconv1d_t<float, float, false>(g, off, map, total_rows, d, K, w, b, out, st);
}

void launch_dwconv1d_post_glu_bf16(const void* g, const int* off, const int* map,
                                   int total_rows, int d, int K, const float* w, const float* b,
                                   void* out, hipStream_t st) {
  launch_glu_dwconv1d_t<__bf16, __bf16, false>(reinterpret_cast<const __bf16*>(g), off, map,
                                               total_rows, d, K, w, b,
                                               reinterpret_cast<__bf16*>(out), st);
}

void launch_glu_dwconv1d(const float* x2, const int* off, const int* map, int total_rows, int d,
                         int K, const float* w, const float* b, float* out, hipStream_t st) {
  launch_glu_dwconv1d_t(x2, off, map, total_rows, d, K, w, b, out, st);
}

void launch_glu_dwconv1d_bf16(const void* x2, const int* off, const int* map, int total_rows,
                              int d, int K, const float* w, const float* b, void* out,
                              hipStream_t st) {
  launch_glu_dwconv1d_t(reinterpret_cast<const __bf16*>(x2), off, map, total_rows, d, K, w, b,
                        reinterpret_cast<__bf16*>(out), st);
}

// =====================================================================================
// SimpleDownsample / SimpleUpsample + bypass, convert_num_channels
// =====================================================================================
struct DsW {
  float w[8];
};

// float4 per thread, 32-bit index math (rows * d / 4 < 2^31 at any batch the engine forms)
// DS = the factor (2, 4, 8): exactly DS loads per output; DS = 0: any factor <= 8 at run time
// (8 loads per output, the ones past ds duplicates)
template <int DS>
__global__ void downsample_kernel(const float* __restrict__ x, const int* __restrict__ off_in,
                                  const int* __restrict__ off_out, const int* __restrict__ map_out,
                                  int total_out,
                                  int d4, int ds, DsW wts, float* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total_out * d4) return;
  const int r = e / d4, c4 = e - r * d4;
  const int b = map_out[r];
  const int tp = r - off_out[b];
  const int base = off_in[b];
  const int L = off_in[b + 1] - base;
  const float4* x4 = reinterpret_cast<const float4*>(x);
  constexpr int NL = DS > 0 ? DS : 8;
  const int f = DS > 0 ? DS : ds;
  float4 xv[NL];
#pragma unroll
  for (int u = 0; u < NL; ++u) {  // all loads in flight
    int t = tp * f + (u < f ? u : 0);
    if (t > L - 1) t = L - 1;  // SimpleDownsample pads with the last frame
    xv[u] = x4[(base + t) * d4 + c4];
  }
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < NL; ++u)
    if (u < f) {
      acc.x = fmaf(wts.w[u], xv[u].x, acc.x);
      acc.y = fmaf(wts.w[u], xv[u].y, acc.y);
      acc.z = fmaf(wts.w[u], xv[u].z, acc.z);
      acc.w = fmaf(wts.w[u], xv[u].w, acc.w);
    }
  reinterpret_cast<float4*>(out)[e] = acc;
}

void launch_downsample(const float* x, const int* off_in, const int* off_out, const int* map_out,
                       int total_out, int d, int ds, const float* w_host8, float* out,
                       hipStream_t st) {
  const long n = (long)total_out * (d / 4);
  if (n <= 0) return;
  ZASR_REQUIRE(d % 4 == 0 && n < (1L << 31), "downsample: width must be a multiple of 4");
  DsW w{};
  for (int i = 0; i < ds && i < 8; ++i) w.w[i] = w_host8[i];
  ZASR_REQUIRE(ds >= 1 && ds <= 8, "downsample: factor must be in [1, 8]");
#define ZASR_DS(DSV) ZASR_LAUNCH((downsample_kernel<DSV>), dim3(cdivl(n, 256)), dim3(256), 0, st, x, off_in, \
                                        off_out, map_out, total_out, d / 4, ds, w, out)
  if (ds == 2) ZASR_DS(2);
  else if (ds == 4) ZASR_DS(4);
  else if (ds == 8) ZASR_DS(8);
  else ZASR_DS(0);
#undef ZASR_DS
}

// The seam between encoder stacks (icefall Zipformer2Encoder / DownsampledZipformer2Encoder,
// 3P): y = orig + (SimpleUpsample(xd) - orig) * s (out_combiner bypass; ds == 1: y = orig),
// written once as
//   * the next stack's input, convert_num_channels'd to width dn (truncate / zero-pad), and
//   * columns [c0, d) of the full-dim encoder output (_get_full_dim_output),
// so the stack output never makes a separate round trip through HBM.  float4 per thread.
__global__ void stack_glue_kernel(const float* __restrict__ xd, const float* __restrict__ orig,
                                  const int* __restrict__ off_in, const int* __restrict__ off_ds,
                                  const int* __restrict__ map_in, int rows, int d4, int ds_shift,
                                  const float* __restrict__ s, float* __restrict__ next, int dn4,
                                  float* __restrict__ full, int ldf4, int c04) {
  const int w4 = d4 > dn4 ? d4 : dn4;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * w4) return;
  const int r = e / w4, c4 = e - r * w4;
  float4 y = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c4 < d4) {
    const float4 o = reinterpret_cast<const float4*>(orig)[r * d4 + c4];
    y = o;
    if (ds_shift > 0) {
      const int b = map_in[r];
      const int t = r - off_in[b];
      const float4 up = reinterpret_cast<const float4*>(xd)[(off_ds[b] + (t >> ds_shift)) * d4 + c4];
      const float4 k = reinterpret_cast<const float4*>(s)[c4];
      y.x = o.x + (up.x - o.x) * k.x;
      y.y = o.y + (up.y - o.y) * k.y;
      y.z = o.z + (up.z - o.z) * k.z;
      y.w = o.w + (up.w - o.w) * k.w;
    }
    if (full != nullptr && c4 >= c04) reinterpret_cast<float4*>(full)[r * ldf4 + c4] = y;
  }
  if (next != nullptr && c4 < dn4) reinterpret_cast<float4*>(next)[r * dn4 + c4] = y;
}

void launch_stack_glue(const float* xd, const float* orig, const int* off_in, const int* off_ds,
                       const int* map_in, int rows, int d, int ds, const float* s, float* next,
                       int dn, float* full, int ldf, int c0, hipStream_t st) {
  const int w = d > dn ? d : dn;
  const long n = (long)rows * (w / 4);
  if (n <= 0) return;
  ZASR_REQUIRE(d % 4 == 0 && dn % 4 == 0 && ldf % 4 == 0 && c0 % 4 == 0 && n < (1L << 31),
               "stack glue: widths must be multiples of 4");
  int shift = 0;
  while ((1 << shift) < ds) ++shift;
  ZASR_REQUIRE((1 << shift) == ds, "stack glue: downsampling factor must be a power of 2");
  ZASR_LAUNCH(stack_glue_kernel, dim3(cdivl(n, 256)), dim3(256), 0, st, xd, orig, off_in,
                     off_ds, map_in, rows, d / 4, shift, s, next, dn / 4, full, ldf / 4, c0 / 4);
}

__global__ void upsample_combine_kernel(const float* __restrict__ xd,
                                        const float* __restrict__ orig,
                                        const int* __restrict__ off_in,
                                        const int* __restrict__ off_ds,
                                        const int* __restrict__ map_in, int total_rows, int d,
                                        int ds,
                                        const float* __restrict__ s, float* __restrict__ y) {
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)total_rows * d) return;
  int r = (int)(e / d), c = (int)(e - (long)r * d);
  int b = map_in[r];
  int t = r - off_in[b];
  float up = xd[(long)(off_ds[b] + t / ds) * d + c];
  float o = orig[e];
  y[e] = o + (up - o) * s[c];
}

void launch_upsample_combine(const float* xd, const float* orig, const int* off_in,
                             const int* off_ds, const int* map_in, int total_rows, int d, int ds,
                             const float* s, float* y, hipStream_t st) {
  long n = (long)total_rows * d;
  if (n <= 0) return;
  ZASR_LAUNCH(upsample_combine_kernel, dim3(cdivl(n, 256)), dim3(256), 0, st, xd, orig,
                     off_in, off_ds, map_in, total_rows, d, ds, s, y);
}

__global__ void copy_cols_kernel(const float* __restrict__ src, int lds, int c0,
                                 float* __restrict__ dst, int ldd, int d0, int ncols, long rows,
                                 int zero_rest, int dst_width) {
  int width = zero_rest ? dst_width : ncols;
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * width) return;
  long r = e / width;
  int c = (int)(e - r * width);
  float v = (c < ncols) ? src[r * lds + c0 + c] : 0.f;
  dst[r * ldd + d0 + c] = v;
}

void launch_copy_cols(const float* src, int lds, int c0, float* dst, int ldd, int d0, int ncols,
                      long rows, bool zero_rest, int dst_width, hipStream_t st) {
  int width = zero_rest ? dst_width : ncols;
  long n = rows * width;
  if (n <= 0) return;
  ZASR_LAUNCH(copy_cols_kernel, dim3(cdivl(n, 256)), dim3(256), 0, st, src, lds, c0, dst,
                     ldd, d0, ncols, rows, zero_rest ? 1 : 0, dst_width);
}

// =====================================================================================
// Attention weights: S[i][j] = q_i . k_j (32 dims, f32 MFMA 32x32x2) + p_i . R[j - i] (4 dims),
// softmax over j < L.  Block = 4 waves = 32 query rows of one (sequence, head); waves stride
// over 32-key blocks.  Pass 1: per-lane online (max, sum) merged across lanes and waves.
// Pass 2: recompute scores and write normalised weights A[h][i][j] (row stride lda = L4).
// =====================================================================================
__global__ __launch_bounds__(256) void attn_softmax_kernel(AttnArgs a) {
  const int b = blockIdx.y;
  const int h = blockIdx.z;
  const int r0 = a.row_off[b];
  const int L = a.row_off[b + 1] - r0;
  const int i0 = blockIdx.x * 32;
  if (i0 >= L) return;
  const int H = a.H;
  const int ldq = 68 * H;
  const int lda = (L + 3) & ~3;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int hl = lane >> 5;
  const int col = lane & 31;

  __shared__ float sQ[32][33];   // [k][i]
  __shared__ float sP[32][4];    // pos query of row i
  __shared__ float sM[4][32], sS[4][32];
  __shared__ float fM[32], fInv[32];

  for (int e = threadIdx.x; e < 32 * 32; e += 256) {
    int i = e >> 5, k = e & 31;
    float v = 0.f;
    if (i0 + i < L) v = a.qkp[(long)(r0 + i0 + i) * ldq + h * 32 + k];
    sQ[k][i] = v;
  }
  if (threadIdx.x < 128) {
    int i = threadIdx.x >> 2, c = threadIdx.x & 3;
    float v = 0.f;
    if (i0 + i < L) v = a.qkp[(long)(r0 + i0 + i) * ldq + 64 * H + h * 4 + c];
    sP[i][c] = v;
  }
  __syncthreads();

  const float* kbase = a.qkp + (long)r0 * ldq + 32 * H + h * 32;
  const float* pos = a.pos_tab + h * 4;
  const int ldp = 4 * H;
  const int nkb = (L + 31) / 32;

  auto scores = [&](int j0, f32x16& acc) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int j = j0 + col;
    float kreg[16];
    if (j < L) {
      const float4* kp = reinterpret_cast<const float4*>(kbase + (long)j * ldq + 16 * hl);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 v = kp[q];
        kreg[4 * q] = v.x;
        kreg[4 * q + 1] = v.y;
        kreg[4 * q + 2] = v.z;
        kreg[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) kreg[q] = 0.f;
    }
    // MFMA step s: lane half hl covers k = 16*hl + s (A: Q[i][k], B: K[j][k])
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      float av = sQ[16 * hl + s][col];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, kreg[s], acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * hl;
      const int x = j - (i0 + i);
      const float4 pr = *reinterpret_cast<const float4*>(pos + (long)(x + a.pmax - 1) * ldp);
      float ps = sP[i][0] * pr.x;
      ps = fmaf(sP[i][1], pr.y, ps);
      ps = fmaf(sP[i][2], pr.z, ps);
      ps = fmaf(sP[i][3], pr.w, ps);
      acc[r] = (j < L) ? acc[r] + ps : -INFINITY;
    }
  };

  float m[16], l[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
  for (int kb = wid; kb < nkb; kb += 4) {
    f32x16 acc;
    scores(kb * 32, acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float s = acc[r];
      if (s == -INFINITY) continue;
      if (s > m[r]) {
        l[r] = l[r] * expf(m[r] - s) + 1.f;
        m[r] = s;
      } else {
        l[r] += expf(s - m[r]);
      }
    }
  }
  // merge over the 32 lanes sharing a row
#pragma unroll
  for (int r = 0; r < 16; ++r) {
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      float om = __shfl_xor(m[r], o, 64);
      float ol = __shfl_xor(l[r], o, 64);
      float nm = fmaxf(m[r], om);
      float nl = 0.f;
      if (m[r] != -INFINITY) nl += l[r] * expf(m[r] - nm);
      if (om != -INFINITY) nl += ol * expf(om - nm);
      m[r] = nm;
      l[r] = nl;
    }
    if (col == 0) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * hl;
      sM[wid][i] = m[r];
      sS[wid][i] = l[r];
    }
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int i = threadIdx.x;
    float mm = -INFINITY;
    for (int w = 0; w < 4; ++w) mm = fmaxf(mm, sM[w][i]);
    float ss = 0.f;
    for (int w = 0; w < 4; ++w)
      if (sM[w][i] != -INFINITY) ss += sS[w][i] * expf(sM[w][i] - mm);
    fM[i] = mm;
    fInv[i] = 1.f / ss;
    if (i0 + i < L) {
      float* sp = a.stats + ((long)(r0 + i0 + i) * H + h) * 2;
      sp[0] = mm;
      sp[1] = 1.f / ss;
    }
  }
  __syncthreads();
  if (h >= a.write_heads) return;
  float* out = a.attn + a.a_off[b] + (long)h * L * lda;
  for (int kb = wid; kb < nkb; kb += 4) {
    f32x16 acc;
    scores(kb * 32, acc);
    const int j = kb * 32 + col;
    if (j >= L) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * hl;
      if (i0 + i >= L) continue;
      out[(long)(i0 + i) * lda + j] = expf(acc[r] - fM[i]) * fInv[i];
    }
  }
}

// =====================================================================================
// Self-attention consumer fused with the score recompute (flash style, no materialised
// weights): per (sequence, 32 queries, head), the 4 waves split the 32-key blocks:
//   S^T = K Q^T + p_i . R[j - i]   (lane = query i, accumulator registers = 16 keys j),
//   P^T = exp(S^T - m_i) / l_i,    O^T += V^T P^T.
// ONLINE: m_i / l_i are running statistics (rescaled per key block, merged over waves at the
// end) and are written out for the second self-attention of the layer; otherwise they come
// from that output.  BF16: QK^T and PV on v_mfma_f32_32x32x16_bf16 (2 + 2 MFMAs per key
// block; the PV k-slots are the S^T accumulator registers as they stand, with V staged in
// the same permuted key order); else exact f32 MFMA 32x32x2 (16 + 16).
// =====================================================================================
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t cvt8(const float4 x0, const float4 x1) {
  bf16x8_t v;
  v[0] = (__bf16)x0.x; v[1] = (__bf16)x0.y; v[2] = (__bf16)x0.z; v[3] = (__bf16)x0.w;
  v[4] = (__bf16)x1.x; v[5] = (__bf16)x1.y; v[6] = (__bf16)x1.z; v[7] = (__bf16)x1.w;
  return v;
}

template <bool ONLINE, bool BF16>
__global__ __launch_bounds__(256) void attn_sa_kernel(AttnSAArgs a) {
  const int b = blockIdx.y;
  const int h = blockIdx.z;
  const int r0 = a.row_off[b];
  const int L = a.row_off[b + 1] - r0;
  const int i0 = blockIdx.x * 32;
  if (i0 >= L) return;
  const int H = a.H;
  const int ldq = 68 * H;
  const int ldv = 12 * H;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = lane & 31, h2 = lane >> 5;
  __shared__ float4 sR[4][64];
  __shared__ float sV[4][32][13];                               // f32 path
  __shared__ __attribute__((aligned(16))) __bf16 sVt[4][12][32];  // bf16 path, permuted keys
  __shared__ float red[3][16][64];
  __shared__ float redM[4][64], redL[4][64];

  const int i = i0 + c;
  const bool iv = i < L;
  const int ic = iv ? i : L - 1;
  const float* qrow = a.qkp + (long)(r0 + ic) * ldq + h * 32;
  float qreg[16];
  bf16x8_t qf[2];
  if constexpr (BF16) {
    const float4* q0 = reinterpret_cast<const float4*>(qrow + 8 * h2);
    const float4* q1 = reinterpret_cast<const float4*>(qrow + 16 + 8 * h2);
    qf[0] = cvt8(q0[0], q0[1]);
    qf[1] = cvt8(q1[0], q1[1]);
  } else {
    const float4* qp = reinterpret_cast<const float4*>(qrow + 16 * h2);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = qp[q];
      qreg[4 * q] = v.x;
      qreg[4 * q + 1] = v.y;
      qreg[4 * q + 2] = v.z;
      qreg[4 * q + 3] = v.w;
    }
  }
  const float4 pq = *reinterpret_cast<const float4*>(a.qkp + (long)(r0 + ic) * ldq + 64 * H + 4 * h);
  float mi = 0.f, li = 0.f;
  if constexpr (!ONLINE) {
    mi = a.stats[((long)(r0 + ic) * H + h) * 2];
    li = a.stats[((long)(r0 + ic) * H + h) * 2 + 1];
  }
  float m_run = -INFINITY, l_run = 0.f;
  const float* kbase = a.qkp + (long)r0 * ldq + 32 * H + h * 32;
  const float* vbase = a.v + (long)r0 * ldv + 12 * h;
  const int nkb = (L + 31) / 32;

  f32x16 o;
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  for (int kb = wid; kb < nkb; kb += 4) {
    const int j0 = kb * 32;
    // pos rows x = j0 - i0 - 31 + l, l < 63 (loads unconditional, clamped: a guarded load
    // becomes a branch with its own vmcnt(0) wait)
    {
      const int x = j0 - i0 - 31 + (lane < 63 ? lane : 62);
      const float4 pr = *reinterpret_cast<const float4*>(a.pos_tab + (long)(x + a.pmax - 1) * 4 * H + 4 * h);
      if (lane < 63) sR[wid][lane] = pr;
    }
    // values of this key block: 32 rows x 12
    float4 vv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = lane + 64 * u;
      const int jj = (e < 96 ? e : 95) / 3, q = (e < 96 ? e : 95) - jj * 3;
      const int jr = j0 + jj < L ? j0 + jj : L - 1;
      vv[u] = *reinterpret_cast<const float4*>(vbase + (long)jr * ldv + 4 * q);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = lane + 64 * u;
      if (e >= 96) continue;
      const int jj = e / 3, q = e - jj * 3;
      float4 v = j0 + jj < L ? vv[u] : make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (BF16) {
        // key jj sits in accumulator register r = (jj&3) + 4*(jj>>3) of lane half (jj>>2)&1;
        // MFMA m = r >> 3 takes it in k-slot 8 * half + (r & 7)
        const int r = (jj & 3) + 4 * (jj >> 3);
        const int slot = 16 * (r >> 3) + 8 * ((jj >> 2) & 1) + (r & 7);
        sVt[wid][4 * q][slot] = (__bf16)v.x;
        sVt[wid][4 * q + 1][slot] = (__bf16)v.y;
        sVt[wid][4 * q + 2][slot] = (__bf16)v.z;
        sVt[wid][4 * q + 3][slot] = (__bf16)v.w;
      } else {
        sV[wid][jj][4 * q] = v.x;
        sV[wid][jj][4 * q + 1] = v.y;
        sV[wid][jj][4 * q + 2] = v.z;
        sV[wid][jj][4 * q + 3] = v.w;
      }
    }
    const int j = j0 + c;
    f32x16 sc;
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[r] = 0.f;
    if constexpr (BF16) {
      // keys past L are masked to -inf below, so their (clamped) values do not matter
      const int jc = j < L ? j : L - 1;
      const float4* k0 = reinterpret_cast<const float4*>(kbase + (long)jc * ldq + 8 * h2);
      const float4* k1 = reinterpret_cast<const float4*>(kbase + (long)jc * ldq + 16 + 8 * h2);
      const bf16x8_t kf0 = cvt8(k0[0], k0[1]);
      const bf16x8_t kf1 = cvt8(k1[0], k1[1]);
      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf0, qf[0], sc, 0, 0, 0);
      sc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf1, qf[1], sc, 0, 0, 0);
    } else {
      float kreg[16];
      {
        const int jc = j < L ? j : L - 1;  // masked below
        const float4* kp = reinterpret_cast<const float4*>(kbase + (long)jc * ldq + 16 * h2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 v = kp[q];
          kreg[4 * q] = v.x;
          kreg[4 * q + 1] = v.y;
          kreg[4 * q + 2] = v.z;
          kreg[4 * q + 3] = v.w;
        }
      }
#pragma unroll
      for (int s = 0; s < 16; ++s) sc = __builtin_amdgcn_mfma_f32_32x32x2f32(kreg[s], qreg[s], sc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jr = (r & 3) + 8 * (r >> 2) + 4 * h2;
      const float4 pr = sR[wid][jr - c + 31];
      float ps = pq.x * pr.x;
      ps = fmaf(pq.y, pr.y, ps);
      ps = fmaf(pq.z, pr.z, ps);
      ps = fmaf(pq.w, pr.w, ps);
      sc[r] = (j0 + jr < L && iv) ? sc[r] + ps : -INFINITY;
    }
    if constexpr (ONLINE) {
      float bm = sc[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) bm = fmaxf(bm, sc[r]);
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m_run, bm);
      if (mn != -INFINITY) {
        const float scale = __expf(m_run - mn);  // m_run = -inf -> 0
        l_run *= scale;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          o[r] *= scale;
          sc[r] = __expf(sc[r] - mn);
          l_run += sc[r];
        }
        m_run = mn;
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) sc[r] = 0.f;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) sc[r] = __expf(sc[r] - mi) * li;  // -inf -> 0
    }
    if constexpr (BF16) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        bf16x8_t pf, vf;
#pragma unroll
        for (int t = 0; t < 8; ++t) pf[t] = (__bf16)sc[8 * m + t];
        if (c < 12) {
          vf = *reinterpret_cast<const bf16x8_t*>(&sVt[wid][c][16 * m + 8 * h2]);
        } else {
#pragma unroll
          for (int t = 0; t < 8; ++t) vf[t] = (__bf16)0.f;
        }
        o = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jr = (r & 3) + 8 * (r >> 2) + 4 * h2;
        const float av = c < 12 ? sV[wid][jr][c] : 0.f;
        o = __builtin_amdgcn_mfma_f32_32x32x2f32(av, sc[r], o, 0, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr (ONLINE) {
    // this wave's row statistics: both lane halves hold the same max, partial sums
    l_run += __shfl_xor(l_run, 32, 64);
    redM[wid][lane] = m_run;
    redL[wid][lane] = l_run;
  }
  if (wid > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wid - 1][r][lane] = o[r];
  }
  __syncthreads();
  if (wid == 0 && iv) {
    float wsc[4] = {1.f, 1.f, 1.f, 1.f};
    float inv = 1.f;
    if constexpr (ONLINE) {
      float M = redM[0][lane];
      for (int w = 1; w < 4; ++w) M = fmaxf(M, redM[w][lane]);
      float Ls = 0.f;
      for (int w = 0; w < 4; ++w) {
        wsc[w] = redM[w][lane] == -INFINITY ? 0.f : __expf(redM[w][lane] - M);
        Ls += redL[w][lane] * wsc[w];
      }
      inv = 1.f / Ls;
      if (h2 == 0) {
        float* sp = a.stats_out + ((long)(r0 + i) * H + h) * 2;
        sp[0] = M;
        sp[1] = inv;
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int v = (r & 3) + 8 * (r >> 2) + 4 * h2;
      if (v < 12) {
        float acc = o[r] * wsc[0] + red[0][r][lane] * wsc[1] + red[1][r][lane] * wsc[2] +
                    red[2][r][lane] * wsc[3];
        a.out[(long)(r0 + i) * ldv + 12 * h + v] = acc * inv;
      }
    }
  }
}

void launch_attn_sa(const AttnSAArgs& a, bool online, bool bf16, hipStream_t st) {
  if (a.nseq <= 0 || a.max_len <= 0) return;
  dim3 grid(cdiv(a.max_len, 32), a.nseq, a.H);
  if (online && bf16) ZASR_LAUNCH((attn_sa_kernel<true, true>), grid, dim3(256), 0, st, a);
  else if (online) ZASR_LAUNCH((attn_sa_kernel<true, false>), grid, dim3(256), 0, st, a);
  else if (bf16) ZASR_LAUNCH((attn_sa_kernel<false, true>), grid, dim3(256), 0, st, a);
  else ZASR_LAUNCH((attn_sa_kernel<false, false>), grid, dim3(256), 0, st, a);
}

void launch_attn_softmax(const AttnArgs& a, hipStream_t st) {
  if (a.nseq <= 0 || a.max_len <= 0) return;
  dim3 grid(cdiv(a.max_len, 32), a.nseq, a.write_heads < a.H ? a.write_heads : a.H);
  ZASR_LAUNCH(attn_softmax_kernel, grid, dim3(256), 0, st, a);
}

}  // namespace zasr
