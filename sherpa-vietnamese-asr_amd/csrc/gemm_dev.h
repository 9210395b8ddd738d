// Device-side helpers shared by the GEMM translation units (gemm.hip, gemm_x3.hip).
#pragma once
#include "common.h"
#include "gemm.h"

namespace zasr {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// A operand, 4 consecutive k of row gm.  Loads are unconditional (clamped into the valid
// range, zero selected afterwards): a guarded load compiles to a branch with a vmcnt(0) wait,
// which serialises the tile's memory round trips.  Requires M >= 1 and K % 4 == 0.
template <int ALOAD>
__device__ __forceinline__ float4 load_a4(const GemmParams& p, const float* A, int M, int K,
                                          int lda, int gm, int gk) {
  const bool ok = gm < M && gk < K;
  const int m = gm < M ? gm : M - 1;
  const int k = gk < K ? gk : K - 4;
  float4 v;
  if constexpr (ALOAD == ALOAD_DENSE) {
    v = *reinterpret_cast<const float4*>(A + (long)m * lda + k);
  } else if constexpr (ALOAD == ALOAD_CONV2) {
    // out (t, f) of conv.4; k = (kt*3 + kf)*8 + c over conv1 output [T1][80][8]
    const int t = m / 39, f = m - t * 39;
    const int kk = k >> 3, c = k & 7;
    const int kt = kk / 3, kf = kk - kt * 3;
    v = *reinterpret_cast<const float4*>(A + ((long)(2 * t + kt) * 80 + 2 * f + kf) * 8 + c);
  } else if constexpr (ALOAD == ALOAD_CONV3) {
    // out (t, f) of conv.7; k = (kt*3 + kf)*32 + c over conv2 output [L2][39][32]
    const int t = m / 19, f = m - t * 19;
    const int kk = k >> 5, c = k & 31;
    const int kt = kk / 3, kf = kk - kt * 3;
    v = *reinterpret_cast<const float4*>(A + ((long)(t + kt) * 39 + 2 * f + kf) * 32 + c);
  } else if constexpr (ALOAD == ALOAD_BNRELU) {
    v = *reinterpret_cast<const float4*>(A + (long)m * lda + k);
    const float4 s = *reinterpret_cast<const float4*>(p.a_scale + k);
    const float4 b = *reinterpret_cast<const float4*>(p.a_shift + k);
    v = make_float4(fmaxf(fmaf(v.x, s.x, b.x), 0.f), fmaxf(fmaf(v.y, s.y, b.y), 0.f),
                    fmaxf(fmaf(v.z, s.z, b.z), 0.f), fmaxf(fmaf(v.w, s.w, b.w), 0.f));
  } else {  // ALOAD_IM2COL1D
    const GemmIm2col1d& g = p.i2c;
    const int n = m / g.Tout, t = m - n * g.Tout;
    const int q = k / g.C, c = k - q * g.C;
    const int ts = t * g.stride + q * g.dil - g.pad;
    const bool in = ts >= 0 && ts < g.Tin;
    v = *reinterpret_cast<const float4*>(A + ((long)n * g.Tin + (in ? ts : 0)) * lda + c);
    return (ok && in) ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  return ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
}

// logical tile of this block (see header comment): XCD x owns tiles [x*per + min(x, rem) ...)
__device__ __forceinline__ int xcd_tile(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7;
  const int xcd = b & 7, slot = b >> 3;
  return xcd < rem ? xcd * (per + 1) + slot : rem * (per + 1) + (xcd - rem) * per + slot;
}

// ---- split-bf16 helpers (the bf16x3 / bf16x6 modes) ----
template <int NP>
__device__ __forceinline__ void split_f8(const float (&v)[8], bf16x8 (&pc)[NP]) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float r = v[q];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      const __bf16 h = (__bf16)r;
      pc[t][q] = h;
      if (t + 1 < NP) r -= (float)h;
    }
  }
}

// ---- fp16 hi + scaled-lo pieces (the "f16x3" mode) ----
// x = hi + lo * 2^-11 with hi = fp16(x), lo = fp16((x - hi) * 2^11): 11 + 11 significant bits
// (~2^-22 relative; the residual is exact in f32 and its scaled value stays in the fp16 normal
// range wherever hi does).  A product is hi*hi + (hi*lo + lo*hi) * 2^-11: three fp16 MFMAs at
// the bf16 rate, two accumulators.  Operands must stay below 65504 in magnitude.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr float kF16Lo = 2048.f;
constexpr float kF16LoInv = 1.f / 2048.f;

__device__ __forceinline__ void split_h8(const float (&v)[8], bf16x8 (&pc)[2]) {
  f16x8 h, l;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    h[q] = (_Float16)v[q];
    l[q] = (_Float16)((v[q] - (float)h[q]) * kF16Lo);
  }
  pc[0] = __builtin_bit_cast(bf16x8, h);
  pc[1] = __builtin_bit_cast(bf16x8, l);
}

// FMT 0: NP bf16 pieces (split_f8); FMT 1: the two fp16 pieces (split_h8, NP = 2)
template <int FMT, int NP>
__device__ __forceinline__ void split_fx(const float (&v)[8], bf16x8 (&pc)[NP]) {
  if constexpr (FMT == 1) {
    static_assert(NP == 2, "fp16 format: two pieces");
    split_h8(v, pc);
  } else {
    split_f8<NP>(v, pc);
  }
}

// hi += x0 y0; lo += x1 y0 + x0 y1 (fp16 MFMAs; pieces carried in bf16x8 containers)
__device__ __forceinline__ void mfma_h3(const bf16x8 (&x)[2], const bf16x8 (&y)[2], f32x16& hi,
                                        f32x16& lo) {
  const f16x8 x0 = __builtin_bit_cast(f16x8, x[0]), x1 = __builtin_bit_cast(f16x8, x[1]);
  const f16x8 y0 = __builtin_bit_cast(f16x8, y[0]), y1 = __builtin_bit_cast(f16x8, y[1]);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, y0, lo, 0, 0, 0);
  lo = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, y1, lo, 0, 0, 0);
  hi = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, y0, hi, 0, 0, 0);
}

// acc += sum over u + v < NP of x[u] * y[v], smallest terms first (written out: every index
// a constant, so the piece arrays stay in registers)
template <int NP>
__device__ __forceinline__ f32x16 mfma_split(const bf16x8 (&x)[NP], const bf16x8 (&y)[NP], f32x16 acc) {
#define ZASR_MF(u, v) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x[u], y[v], acc, 0, 0, 0)
  if constexpr (NP == 3) {
    ZASR_MF(2, 0); ZASR_MF(1, 1); ZASR_MF(0, 2);
  }
  if constexpr (NP >= 2) {
    ZASR_MF(NP - 1 == 1 ? 1 : 1, 0); ZASR_MF(0, 1);
  }
  ZASR_MF(0, 0);
#undef ZASR_MF
  return acc;
}

}  // namespace zasr
