// ConvNeXt block of Conv2dSubsampling in the bf16 mode (icefall subsampling.py ConvNeXt, 3P;
// runs inside the reference's exported encoder, core/asr_engine.py:1045-1049):
//
//   out = x + pw2(SwooshL(pw1(dwconv7x7(x) + b_dw) + b1)) + b2
//
// x, out: [rows (50 Hz frames, packed over sequences)][19 freq][128 ch] bf16.  Two kernels:
//
// 1. convnext_dw_kernel: depthwise 7x7 with zero padding outside each frame's own sequence
//    (time) and outside [0, 19) (freq).  Tile = 16 frames x 19 freq x 64 channels with a
//    3-frame halo staged in LDS (bf16, 53.5 KB: two blocks per CU, one staging while the
//    other computes).  A thread owns a channel pair (packed f32 FMAs, weights in registers)
//    and 8 consecutive frames of one freq: every staged value read from LDS feeds up to 7
//    output frames.  Output y = dwconv + bias in bf16.
// 2. convnext_mlp_kernel: 128 positions (frame, freq) per block; the 384-wide hidden layer
//    is produced in three 128-wide slices, each living only in LDS: H^T = W1 Y^T on
//    v_mfma_f32_32x32x16_bf16 (so one lane holds 4 consecutive hidden units of one position
//    per register group: 8-byte LDS stores), SwooshL, then O^T += W2 H^T.  Epilogue adds b2
//    and the residual x and writes bf16.
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace zasr {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kDwT = 16;                // output frames per block
constexpr int kDwH = kDwT + 6;          // staged frames
constexpr int kDwC = 64;                // channels per block

}  // namespace

// staged tile: [kDwH frames][25 = 3 + 19 + 3 freq, zero columns at the edges][kDwC] bf16
constexpr int kDwF = 25;

template <bool MASKED, typename T = __bf16, int C = kDwC>
__device__ __forceinline__ void dw_item(const T* __restrict__ tile, int seg, int f, int p,
                                        const float2 (&w)[49], float2 bias, const int* sLo,
                                        const int* sHi, float2 (&acc)[8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = bias;
  const T* base = tile + ((seg * 8) * kDwF + f) * C + 2 * p;
#pragma unroll
  for (int rr = 0; rr < 14; ++rr) {  // staged frame seg*8 + rr <-> tap row rr - i
    float2 v[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {  // freq tap j <-> staged column f + j
      if constexpr (std::is_same<T, float>::value) {
        v[j] = *reinterpret_cast<const float2*>(base + (rr * kDwF + j) * C);
      } else {
        const bf16x2 hv = *reinterpret_cast<const bf16x2*>(base + (rr * kDwF + j) * C);
        v[j] = make_float2((float)hv[0], (float)hv[1]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ti = rr - i;
      if (ti < 0 || ti > 6) continue;
      if (MASKED) {
        const int dt = ti - 3;
        if (dt < sLo[seg * 8 + i] || dt > sHi[seg * 8 + i]) continue;
      }
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        acc[i].x = fmaf(w[ti * 7 + j].x, v[j].x, acc[i].x);
        acc[i].y = fmaf(w[ti * 7 + j].y, v[j].y, acc[i].y);
      }
    }
    // keep each frame's 7 LDS reads next to their FMAs (hoisting all 98 reads spills)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// T = __bf16 (the bf16 mode, C = 64 channels per block) or float (the f32 / split modes,
// C = 32: the same 16-byte pieces per staged row, 70 KB of LDS); the f32 variant replaces a
// one-output-per-thread kernel that re-read every staged value 49 times (7 ms per hour).
template <typename T = __bf16, int C = kDwC>
__global__ __launch_bounds__(256) void convnext_dw_kernel(
    const T* __restrict__ x, const int* __restrict__ L_off, const int* __restrict__ L_map,
    int total_rows, const float* __restrict__ dw_w, const float* __restrict__ dw_b,
    T* __restrict__ y) {
  constexpr int PAIRS = C / 2;          // channel pairs per block
  constexpr int EPP = 16 / sizeof(T);   // elements per 16-byte piece
  constexpr int PPR = C / EPP;          // pieces per staged (frame, freq) row
  static_assert(PPR == 8, "eight 16-byte pieces per row");
  typedef T T8 __attribute__((ext_vector_type(EPP)));
  __shared__ __attribute__((aligned(16))) T tile[kDwH * kDwF * C];
  // the weights pass through the tile's storage before the tile is written (C * 49 floats fit)
  float* const sW = reinterpret_cast<float*>(tile);
  static_assert(C * 49 * 4 <= (int)sizeof(tile), "weights staged in the tile buffer");
  __shared__ int sLo[kDwT], sHi[kDwT], sMasked;
  const int t0 = blockIdx.x * kDwT;
  const int c0 = blockIdx.y * C;
  const int tid = threadIdx.x;
  if (tid == 0) sMasked = 0;
  // every global load of the block is issued before the first wait: the block's channel
  // weights (staged through LDS with coalesced loads: per-thread loads of its own channels'
  // rows of dw_w [128][49] would touch one cache line per lane and instruction), the bias,
  // the sequence bounds of the tile frames (L_map -> L_off) and the staged input -- one memory
  // round trip
  const int p = tid & (PAIRS - 1);  // channel pair c0 + 2p, c0 + 2p + 1 (fixed per thread)
  constexpr int kWIt = (C * 49 + 255) / 256;
  float wl[kWIt];
#pragma unroll
  for (int q = 0; q < kWIt; ++q) {
    const int i = tid + 256 * q;
    wl[q] = dw_w[c0 * 49 + (i < C * 49 ? i : C * 49 - 1)];
  }
  const float2 bias = make_float2(dw_b[c0 + 2 * p], dw_b[c0 + 2 * p + 1]);
  int seq_lo = 0, seq_hi = 0;
  if (tid < kDwT && t0 + tid < total_rows) {
    const int b = L_map[t0 + tid];
    seq_lo = L_off[b];
    seq_hi = L_off[b + 1];
  }
  // ---- stage frames t0-3 .. t0+18, channels c0..c0+C-1: 22 x 19 x 8 16-byte pieces ----
  constexpr int kPieces = kDwH * 19 * 8;  // 3344
  constexpr int kIt = (kPieces + 255) / 256;
  T8 v[kIt];
#pragma unroll
  for (int k = 0; k < kIt; ++k) {
    const int e = tid + 256 * k;
    const int ec = e < kPieces ? e : kPieces - 1;
    const int rf = ec >> 3, q = ec & 7;
    const int rr = rf / 19, f = rf - rr * 19;
    int r = t0 - 3 + rr;
    const bool ok = e < kPieces && r >= 0 && r < total_rows;
    r = r < 0 ? 0 : (r >= total_rows ? total_rows - 1 : r);
    v[k] = *reinterpret_cast<const T8*>(x + ((long)r * 19 + f) * 128 + c0 + EPP * q);
    if (!ok) {
#pragma unroll
      for (int t = 0; t < EPP; ++t) v[k][t] = (T)0.f;
    }
  }
  // ---- the weights: loads in flight -> LDS -> this thread's channel pair ----
#pragma unroll
  for (int q = 0; q < kWIt; ++q) {
    const int i = tid + 256 * q;
    if (i < C * 49) sW[i] = wl[q];
  }
  __syncthreads();
  float2 w[49];
#pragma unroll
  for (int k = 0; k < 49; ++k) w[k] = make_float2(sW[2 * p * 49 + k], sW[(2 * p + 1) * 49 + k]);
  __syncthreads();  // every thread holds its weights before the tile overwrites them
  // ---- zero freq padding columns (3 + 3 per staged frame, 8 pieces of 16 B each) ----
  for (int e = tid; e < kDwH * 6 * 8; e += 256) {
    const int q = e & 7, cf = (e >> 3) % 6, rr = (e >> 3) / 6;
    const int fcol = cf < 3 ? cf : 19 + cf;
    T8 z;
#pragma unroll
    for (int t = 0; t < EPP; ++t) z[t] = (T)0.f;
    *reinterpret_cast<T8*>(tile + (rr * kDwF + fcol) * C + EPP * q) = z;
  }
#pragma unroll
  for (int k = 0; k < kIt; ++k) {
    const int e = tid + 256 * k;
    if (e < kPieces) {
      const int rf = e >> 3, q = e & 7;
      const int rr = rf / 19, f = rf - rr * 19;
      *reinterpret_cast<T8*>(tile + (rr * kDwF + 3 + f) * C + EPP * q) = v[k];
    }
  }
  if (tid < kDwT) {
    const int r = t0 + tid;
    int lo = -3, hi = 3;
    if (r < total_rows) {
      lo = max(seq_lo - r, -3);
      hi = min(seq_hi - 1 - r, 3);
    }
    sLo[tid] = lo;
    sHi[tid] = hi;
  }
  __syncthreads();
  if (tid < kDwT && (sLo[tid] != -3 || sHi[tid] != 3)) atomicOr(&sMasked, 1);
  __syncthreads();

  const bool masked = sMasked != 0;
  constexpr int kItems = 2 * 19 * PAIRS;  // (segment, freq, channel pair) work items
  for (int it = tid; it < kItems; it += 256) {
    const int q = it / PAIRS;  // (segment, freq)
    const int seg = q / 19, f = q - seg * 19;
    float2 acc[8];
    if (masked)
      dw_item<true, T, C>(tile, seg, f, p, w, bias, sLo, sHi, acc);
    else
      dw_item<false, T, C>(tile, seg, f, p, w, bias, sLo, sHi, acc);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = t0 + seg * 8 + i;
      if (r < total_rows) {
        if constexpr (std::is_same<T, float>::value) {
          *reinterpret_cast<float2*>(y + ((long)r * 19 + f) * 128 + c0 + 2 * p) = acc[i];
        } else {
          bf16x2 o;
          o[0] = (__bf16)acc[i].x;
          o[1] = (__bf16)acc[i].y;
          *reinterpret_cast<bf16x2*>(y + ((long)r * 19 + f) * 128 + c0 + 2 * p) = o;
        }
      }
    }
  }
}

void launch_dwconv2d_tiled(const float* x, const int* L_off, const int* L_map, int total_rows,
                           const float* w, const float* b, float* out, hipStream_t st) {
  if (total_rows <= 0) return;
  ZASR_LAUNCH((convnext_dw_kernel<float, 32>), dim3(cdiv(total_rows, kDwT), 128 / 32),
                     dim3(256), 0, st, x, L_off, L_map, total_rows, w, b, out);
}

// =====================================================================================
// pointwise MLP + residual.  Y / H tiles in LDS: [128 positions][136] bf16 (272-byte rows:
// conflict-free 16-byte fragment reads).  Wave w owns hidden (pw1) / output (pw2) columns
// 32 w .. 32 w + 31 of each 128-wide slice, for all 128 positions (4 MFMA tiles).
// W1 / W2 arrive in MFMA-fragment order (pack_frag32_host: one contiguous 1 KB wave read per
// fragment), b1 is staged in LDS, and the slice barriers are LDS-only, so the weight
// prefetches stay in flight across them.
// =====================================================================================
namespace {
__device__ __forceinline__ void lds_barrier_cx() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}
}  // namespace

// W [rows][cols] bf16 -> [rows/32][cols/16][64 lanes][8]: element j of lane l of fragment
// (g, s) is W[32 g + (l & 31)][16 s + 8 (l >> 5) + j] (v_mfma_f32_32x32x16_bf16 A operand)
void pack_frag32_host(const __bf16* w, int rows, int cols, __bf16* out) {
  for (int g = 0; g < rows / 32; ++g)
    for (int s = 0; s < cols / 16; ++s)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j)
          out[(((size_t)g * (cols / 16) + s) * 64 + l) * 8 + j] =
              w[(size_t)(32 * g + (l & 31)) * cols + 16 * s + 8 * (l >> 5) + j];
}
namespace {
constexpr int kMlpM = 128;
constexpr int kMlpLd = 136;
}  // namespace

__global__ __launch_bounds__(256, 2) void convnext_mlp_kernel(
    const __bf16* __restrict__ yin, const __bf16* __restrict__ x, long npos,
    const __bf16* __restrict__ w1, const float* __restrict__ b1, const __bf16* __restrict__ w2,
    const float* __restrict__ b2, __bf16* __restrict__ out) {
  // Y and H tiles in one array: the epilogue stages O + b2 over both
  __shared__ __attribute__((aligned(16))) __bf16 YH[2 * kMlpM * kMlpLd];
  __bf16* const Ys = YH;
  __bf16* const Hs = YH + kMlpM * kMlpLd;
  __shared__ float sB1[384];
  const long p0 = (long)blockIdx.x * kMlpM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int col = lane & 31, half = lane >> 5;
  // ---- Y tile: 128 x 128 bf16 = 2048 16-byte pieces, 8 per thread ----
  {
    bf16x8 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = tid + 256 * k;
      long pp = p0 + (e >> 4);
      pp = pp < npos ? pp : npos - 1;
      v[k] = *reinterpret_cast<const bf16x8*>(yin + pp * 128 + 8 * (e & 15));
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = tid + 256 * k;
      *reinterpret_cast<bf16x8*>(Ys + (e >> 4) * kMlpLd + 8 * (e & 15)) = v[k];
    }
    for (int e = tid; e < 384; e += 256) sB1[e] = b1[e];
  }
  lds_barrier_cx();

  f32x16 acc2[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[t][r] = 0.f;

  // weight fragments straight from L2 (96 KB each, shared by every block): W1 of slice n3 + 1
  // is fetched under slice n3's pw2 MFMAs and W2 of slice n3 under its pw1 MFMAs, so only the
  // first slice's W1 round trip is exposed
  bf16x8 wf1[8], wf2[8];
  // fragment (row group, k-step) of the packed images: W1 [384][128] -> [12][8], W2 [128][384] -> [4][24]
  auto w1frag = [&](int g, int ks) { return *reinterpret_cast<const bf16x8*>(w1 + (((long)g * 8 + ks) * 64 + lane) * 8); };
  auto w2frag = [&](int g, int ks) { return *reinterpret_cast<const bf16x8*>(w2 + (((long)g * 24 + ks) * 64 + lane) * 8); };
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) wf1[ks] = w1frag(wid, ks);
  for (int n3 = 0; n3 < 3; ++n3) {
    // ---- H^T slice: rows = hidden units n3*128 + 32 wid + (0..31), cols = positions ----
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) wf2[ks] = w2frag(wid, n3 * 8 + ks);
    f32x16 acc1[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[t][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 yf =
            *reinterpret_cast<const bf16x8*>(Ys + (t * 32 + col) * kMlpLd + ks * 16 + 8 * half);
        acc1[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf1[ks], yf, acc1[t], 0, 0, 0);
      }
    }
    {  // next slice's W1 (unconditional: a branch here costs exact vmcnt tracking)
      const int nn = n3 < 2 ? n3 + 1 : 2;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) wf1[ks] = w1frag(nn * 4 + wid, ks);
    }
    // bias of the 16 hidden rows this lane holds: wid*32 + (r&3) + 8 (r>>2) + 4 half
    float bb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bb[r] = sB1[n3 * 128 + wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
    if (n3 > 0) lds_barrier_cx();  // the previous slice's pw2 is done reading Hs
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 hv;
#pragma unroll
        for (int e = 0; e < 4; ++e) hv[e] = (__bf16)swooshl_fast(acc1[t][4 * g + e] + bb[4 * g + e]);
        *reinterpret_cast<bf16x4*>(Hs + (t * 32 + col) * kMlpLd + wid * 32 + 8 * g + 4 * half) = hv;
      }
    lds_barrier_cx();
    // ---- O^T += W2[:, slice] H^T: rows = output channels 32 wid + (0..31) ----
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16x8 hf =
            *reinterpret_cast<const bf16x8*>(Hs + (t * 32 + col) * kMlpLd + ks * 16 + 8 * half);
        acc2[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf2[ks], hf, acc2[t], 0, 0, 0);
      }
    }
  }

  // ---- out = x + (O + b2) through LDS: O + b2 staged [position][channel] f32 over the Y / H
  // tiles, then each lane owns 16-byte pieces of whole 256-byte output rows (the fragment layout
  // would store 8-byte pieces of 32 rows per instruction: 1.43 -> 1.25 ms per hour,
  // tools/cnx_lab.hip, bit-identical) ----
  constexpr int OLD = 132;  // f32 row stride: 528 B
  static_assert(kMlpM * OLD * 4 <= 2 * kMlpM * kMlpLd * 2, "O staging fits the Y / H tiles");
  float* Os = reinterpret_cast<float*>(YH);
  bf16x8 xr8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {  // residual pieces in flight under the staging
    const int e = tid + 256 * k;
    long pp = p0 + (e >> 4);
    pp = pp < npos ? pp : npos - 1;
    xr8[k] = *reinterpret_cast<const bf16x8*>(x + pp * 128 + 8 * (e & 15));
  }
  lds_barrier_cx();  // every wave's last pw2 is done reading Hs
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int ch = wid * 32 + 8 * g + 4 * half;
    const float4 bo = *reinterpret_cast<const float4*>(b2 + ch);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float4 v;
      v.x = acc2[t][4 * g + 0] + bo.x;
      v.y = acc2[t][4 * g + 1] + bo.y;
      v.z = acc2[t][4 * g + 2] + bo.z;
      v.w = acc2[t][4 * g + 3] + bo.w;
      *reinterpret_cast<float4*>(Os + (t * 32 + col) * OLD + ch) = v;
    }
  }
  lds_barrier_cx();
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int e = tid + 256 * k, pl = e >> 4, c8 = 8 * (e & 15);
    const long pp = p0 + pl;
    const float4 a = *reinterpret_cast<const float4*>(Os + pl * OLD + c8);
    const float4 b = *reinterpret_cast<const float4*>(Os + pl * OLD + c8 + 4);
    const float ov[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (__bf16)((float)xr8[k][q] + ov[q]);
    if (pp < npos) *reinterpret_cast<bf16x8*>(out + pp * 128 + c8) = o;
  }
}

// =====================================================================================
// f16x3 ConvNeXt MLP: out = x + pw2(SwooshL(pw1(y) + b1)) + b2 in f32 with every product on
// fp16 MFMAs as hi*hi + (hi*lo + lo*hi) * 2^-11 (gemm_dev.h split_h8: f32 quality), the
// 384-wide hidden layer never leaving the CU (the unfused f16x3 path writes and re-reads it in
// f32: 5.8 GB per hour of audio).  Structure of convnext_mlp_kernel: 128 positions per block,
// the hidden layer in three 128-wide slices; Y and the H slice live in LDS as (hi, lo) fp16
// piece images (139 KB: one block per CU, one wave per SIMD -- MFMA work per wave is long
// enough: 576 MFMAs); W1 / W2 pieces come straight from L2 in MFMA-fragment order
// (pack_frag32_host per piece: piece t of W at wp + t * N * K).
// =====================================================================================
namespace {
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void mfma_h3_cx(bf16x8 wh, bf16x8 wl, bf16x8 yh, bf16x8 yl, f32x16& hi,
                                           f32x16& lo) {
  const f16x8 a0 = __builtin_bit_cast(f16x8, wh), a1 = __builtin_bit_cast(f16x8, wl);
  const f16x8 b0 = __builtin_bit_cast(f16x8, yh), b1 = __builtin_bit_cast(f16x8, yl);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b0, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b1, lo, 0, 0, 0);
  hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b0, hi, 0, 0, 0);
}
}  // namespace

__global__ __launch_bounds__(256, 1) void convnext_mlp_h3_kernel(
    const float* __restrict__ yin, const float* __restrict__ x, long npos,
    const __bf16* __restrict__ w1, const float* __restrict__ b1, const __bf16* __restrict__ w2,
    const float* __restrict__ b2, float* __restrict__ out) {
  // [piece][128 positions][kMlpLd] fp16 bits (bf16 containers)
  __shared__ __attribute__((aligned(16))) __bf16 Ys[2][kMlpM * kMlpLd];
  __shared__ __attribute__((aligned(16))) __bf16 Hs[2][kMlpM * kMlpLd];
  __shared__ float sB1[384];
  constexpr long W1P = 384L * 128, W2P = 128L * 384;  // elements per packed piece image
  const long p0 = (long)blockIdx.x * kMlpM;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int col = lane & 31, half = lane >> 5;
  auto w1frag = [&](int pc, int g, int ks) {
    return *reinterpret_cast<const bf16x8*>(w1 + pc * W1P + (((long)g * 8 + ks) * 64 + lane) * 8);
  };
  auto w2frag = [&](int pc, int g, int ks) {
    return *reinterpret_cast<const bf16x8*>(w2 + pc * W2P + (((long)g * 24 + ks) * 64 + lane) * 8);
  };
  // slice 0's W1 set, in flight under the Y tile's loads and split
  bf16x8 wf[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    wf[ks][0] = w1frag(0, wid, ks);
    wf[ks][1] = w1frag(1, wid, ks);
  }
  // ---- Y tile: 128 positions x 128 channels f32 = 2048 groups of 8, 8 per thread ----
  {
    float4 v0[8], v1[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = tid + 256 * k;
      long pp = p0 + (e >> 4);
      pp = pp < npos ? pp : npos - 1;
      const float* src = yin + pp * 128 + 8 * (e & 15);
      v0[k] = *reinterpret_cast<const float4*>(src);
      v1[k] = *reinterpret_cast<const float4*>(src + 4);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = tid + 256 * k;
      f16x8 hh, ll;
      const float v[8] = {v0[k].x, v0[k].y, v0[k].z, v0[k].w, v1[k].x, v1[k].y, v1[k].z, v1[k].w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        hh[q] = (_Float16)v[q];
        ll[q] = (_Float16)((v[q] - (float)hh[q]) * 2048.f);
      }
      const int o = (e >> 4) * kMlpLd + 8 * (e & 15);
      *reinterpret_cast<f16x8*>(Ys[0] + o) = hh;
      *reinterpret_cast<f16x8*>(Ys[1] + o) = ll;
    }
    for (int e = tid; e < 384; e += 256) sB1[e] = b1[e];
  }
  lds_barrier_cx();

  f32x16 acc2[4], acc2l[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc2[t][r] = acc2l[t][r] = 0.f;
  // one weight-fragment set live at a time (two sets + both accumulator pairs spill); the
  // next slice's W1 set is loaded into the W2 registers pw2 has consumed
  for (int n3 = 0; n3 < 3; ++n3) {
    f32x16 acc1[4], acc1l[4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc1[t][r] = acc1l[t][r] = 0.f;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int o = (t * 32 + col) * kMlpLd + ks * 16 + 8 * half;
        mfma_h3_cx(wf[ks][0], wf[ks][1], *reinterpret_cast<const bf16x8*>(Ys[0] + o),
                   *reinterpret_cast<const bf16x8*>(Ys[1] + o), acc1[t], acc1l[t]);
      }
    }
    // this slice's W2 pieces, in flight under the SwooshL / H write
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      wf[ks][0] = w2frag(0, wid, n3 * 8 + ks);
      wf[ks][1] = w2frag(1, wid, n3 * 8 + ks);
    }
    float bb[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) bb[r] = sB1[n3 * 128 + wid * 32 + (r & 3) + 8 * (r >> 2) + 4 * half];
    if (n3 > 0) lds_barrier_cx();  // the previous slice's pw2 is done reading Hs
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f16x4 hh, ll;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = swooshl_fast(acc1[t][4 * g + e] + acc1l[t][4 * g + e] * (1.f / 2048.f) +
                                       bb[4 * g + e]);
          hh[e] = (_Float16)v;
          ll[e] = (_Float16)((v - (float)hh[e]) * 2048.f);
        }
        const int o = (t * 32 + col) * kMlpLd + wid * 32 + 8 * g + 4 * half;
        *reinterpret_cast<f16x4*>(Hs[0] + o) = hh;
        *reinterpret_cast<f16x4*>(Hs[1] + o) = ll;
      }
    lds_barrier_cx();
    const int nn = n3 < 2 ? n3 + 1 : n3;  // (the last slice re-loads its own W1: unused)
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int o = (t * 32 + col) * kMlpLd + ks * 16 + 8 * half;
        mfma_h3_cx(wf[ks][0], wf[ks][1], *reinterpret_cast<const bf16x8*>(Hs[0] + o),
                   *reinterpret_cast<const bf16x8*>(Hs[1] + o), acc2[t], acc2l[t]);
      }
      // W2 set ks is consumed: its registers take the next slice's W1 set ks, in flight
      // under the remaining pw2 MFMAs
      wf[ks][0] = w1frag(0, nn * 4 + wid, ks);
      wf[ks][1] = w1frag(1, nn * 4 + wid, ks);
    }
  }

  // ---- out = x + O + b2 (f32) ----
  float4 xr[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      long pp = p0 + t * 32 + col;
      pp = pp < npos ? pp : npos - 1;
      xr[g][t] = *reinterpret_cast<const float4*>(x + pp * 128 + wid * 32 + 8 * g + 4 * half);
    }
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int ch = wid * 32 + 8 * g + 4 * half;
    const float4 bo = *reinterpret_cast<const float4*>(b2 + ch);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const long pp = p0 + t * 32 + col;
      const int r = 4 * g;
      float4 o;
      o.x = xr[g][t].x + ((acc2[t][r + 0] + acc2l[t][r + 0] * (1.f / 2048.f)) + bo.x);
      o.y = xr[g][t].y + ((acc2[t][r + 1] + acc2l[t][r + 1] * (1.f / 2048.f)) + bo.y);
      o.z = xr[g][t].z + ((acc2[t][r + 2] + acc2l[t][r + 2] * (1.f / 2048.f)) + bo.z);
      o.w = xr[g][t].w + ((acc2[t][r + 3] + acc2l[t][r + 3] * (1.f / 2048.f)) + bo.w);
      if (pp < npos) *reinterpret_cast<float4*>(out + pp * 128 + ch) = o;
    }
  }
}

void launch_convnext_mlp_h3(const float* y, const float* x, long npos, const void* w1p,
                            const float* b1, const void* w2p, const float* b2, float* out,
                            hipStream_t st) {
  if (npos <= 0) return;
  ZASR_LAUNCH(convnext_mlp_h3_kernel, dim3((unsigned)cdivl(npos, kMlpM)), dim3(256), 0, st,
                     y, x, npos, reinterpret_cast<const __bf16*>(w1p), b1,
                     reinterpret_cast<const __bf16*>(w2p), b2, out);
}

void launch_convnext_bf16(const void* x, const int* L_off, const int* L_map, int total_rows,
                          const float* dw_w, const float* dw_b, const void* w1, const float* b1,
                          const void* w2, const float* b2, void* ytmp, void* out,
                          hipStream_t st) {
  if (total_rows <= 0) return;
  const __bf16* xb = reinterpret_cast<const __bf16*>(x);
  __bf16* yb = reinterpret_cast<__bf16*>(ytmp);
  ZASR_LAUNCH((convnext_dw_kernel<__bf16, kDwC>), dim3(cdiv(total_rows, kDwT), 128 / kDwC),
                     dim3(256), 0, st, xb, L_off, L_map, total_rows, dw_w, dw_b, yb);
  const long npos = (long)total_rows * 19;
  ZASR_LAUNCH(convnext_mlp_kernel, dim3((unsigned)cdivl(npos, kMlpM)), dim3(256), 0, st,
                     yb, xb, npos, reinterpret_cast<const __bf16*>(w1), b1,
                     reinterpret_cast<const __bf16*>(w2), b2, reinterpret_cast<__bf16*>(out));
}

}  // namespace zasr
