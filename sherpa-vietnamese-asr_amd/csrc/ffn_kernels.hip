// Fused Zipformer2 FeedforwardModule in the bf16 mode (icefall zipformer.py, 3P; inside the
// reference's exported encoder, core/asr_engine.py:1045-1049):
//
//   X += W2 SwooshL(W1 X + b1) + b2        X: [R][D] f32 (residual stream), W1 [F][D], W2 [D][F]
//
// The hidden activation (F = 3/4 ff .. 5/4 ff wide) never leaves the CU: one wave owns 32
// tokens (the MFMA column = lane), and for every 32-unit hidden chunk
//   H^T = W1_c X^T           v_mfma_f32_32x32x16_bf16, X^T fragments held in registers
//   H^T <- bf16(SwooshL(H^T + b1_c))   in registers
//   O^T += W2_c H^T          the H^T accumulator registers ARE the B operand (k order
//                            permuted: element j of lane half h at k-step s is hidden row
//                            16 s + 8 (j >> 2) + 4 h + (j & 3)); W2_c is staged in LDS in
//                            that order, so its A fragment is one 16-byte LDS read
// Weight chunks (W1_c [32][D], W2_c [D][32], b1_c) are staged in LDS once per block for its
// 4 waves (128 tokens), double-buffered: the next chunk's global loads are in flight while the
// current chunk computes.  Epilogue: X[token][d] += O^T + b2 (f32 read-modify-write).
// Bytes per token: D * 4 read + D * 4 written; the 2 F D bf16 weight bytes are L2-resident.
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.h"
#include "kernels.h"

namespace zasr {

#ifdef ZASR_FFN_STAMPS  // development: per-phase wall clock of block 0 (tools/ffnw_lab.hip)
__device__ long long g_ffn_stamps[4896];
#define FFN_STAMP(i) \
  if (blockIdx.x == 0 && threadIdx.x == 0 && (i) < 4896) g_ffn_stamps[(i)] = clock64();
#else
#define FFN_STAMP(i)
#endif

namespace {

// LDS-only barrier: __syncthreads() also waits for every global load in flight (vmcnt(0)),
// which would drain the weight prefetches at each of the two barriers per chunk
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kTok = 128;  // tokens per block (4 waves x 32)
constexpr int kMaxF = 2048; // ffn_wide_kernel: b1 staged in LDS
constexpr int kW2Ld = 40;  // W2 chunk row stride (bf16): 80 B

// slot of hidden index k (0..31) in a permuted W2 chunk row: swap bits 2 and 3
__device__ __forceinline__ int w2_slot(int k) { return (k & 0x13) | ((k & 4) << 1) | ((k & 8) >> 1); }

// weight fragments by buffer loads: a descriptor over [p, p + bytes) in SGPRs (p and bytes
// wave-uniform); a fragment's byte offset is wave-uniform too (an SGPR operand) and the lane's
// 16 bytes a constant VGPR, so a load needs no 64-bit address arithmetic
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, long bytes) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long)p >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long)hi << 32) | lo), 0, n, 0x00020000);
}
template <typename V>
__device__ __forceinline__ V buf_load16(__amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, 0));
}

}  // namespace

// split barriers (SB, the wide kernels below): cumulative per-wave counters in LDS, polled
__device__ __forceinline__ void lds_wait_ge(int* p, int target) {
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target)
    __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void lds_signal(int* p, int lane) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's H stores / reads are done
  if (lane == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int D>
__global__ __launch_bounds__(256, (D <= 192 ? 2 : 1)) void ffn_fused_kernel(float* __restrict__ X, int R, int F,
                                                           const __bf16* __restrict__ W1,
                                                           const float* __restrict__ b1,
                                                           const __bf16* __restrict__ W2,
                                                           const float* __restrict__ b2,
                                                           const float* __restrict__ byp_orig,
                                                           const float* __restrict__ byp_scale) {
  constexpr int KS = D / 16;     // k-steps of the first product
  constexpr int OT = D / 32;     // output row tiles of the second
  constexpr int W1LD = D + 8;    // W1 chunk row stride (bf16): odd multiple of 16 B
  constexpr int W1P = 32 * D / 8;  // 16-byte pieces of a W1 chunk
  constexpr int W2P = D * 4;       // 16-byte pieces of a W2 chunk (D rows x 64 B)
  constexpr int P1 = (W1P + 255) / 256, P2 = (W2P + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 sW1[2][32 * W1LD];
  __shared__ __attribute__((aligned(16))) __bf16 sW2[2][D * kW2Ld];
  __shared__ float sB1[2][32];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int col = lane & 31, h2 = lane >> 5;
  const int tok = blockIdx.x * kTok + wid * 32 + col;
  const int tokc = tok < R ? tok : R - 1;
  const int nch = (F + 31) / 32;

  // ---- chunk staging (global -> registers -> LDS) ----
  bf16x8 g1[P1], g2[P2];
  float gb = 0.f;
  auto gload = [&](int c) {
#pragma unroll
    for (int i = 0; i < P1; ++i) {
      const int e = tid + 256 * i < W1P ? tid + 256 * i : W1P - 1;  // clamped, unconditional
      const int row = e / (D / 8), k8 = e - row * (D / 8);
      int hr = c * 32 + row;
      hr = hr < F ? hr : F - 1;  // rows past F: any finite value (their W2 columns are 0)
      g1[i] = *reinterpret_cast<const bf16x8*>(W1 + (long)hr * D + 8 * k8);
    }
#pragma unroll
    for (int i = 0; i < P2; ++i) {
      const int e = tid + 256 * i < W2P ? tid + 256 * i : W2P - 1;
      const int row = e >> 2, q = e & 3;
      const int k0 = c * 32 + 8 * q;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(W2 + (long)row * F + (k0 < F ? k0 : 0));
      if (k0 >= F) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (__bf16)0.f;
      }
      g2[i] = v;
    }
    // unconditional (clamped): a guarded load becomes a branch whose vmcnt(0) would wait
    // for the weight loads just issued
    const int bi = c * 32 + (tid & 31);
    const float bv = b1[bi < F ? bi : F - 1];
    gb = bi < F ? bv : 0.f;
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < P1; ++i) {
      const int e = tid + 256 * i;
      if (e < W1P) {
        const int row = e / (D / 8), k8 = e - row * (D / 8);
        *reinterpret_cast<bf16x8*>(&sW1[buf][row * W1LD + 8 * k8]) = g1[i];
      }
    }
#pragma unroll
    for (int i = 0; i < P2; ++i) {
      const int e = tid + 256 * i;
      if (e >= W2P) break;
      const int row = e >> 2, q = e & 3;
      // k = 8 q + m: m = 0..3 -> slot w2_slot(8q), m = 4..7 -> w2_slot(8q + 4)
      bf16x4 lo, hi;
      lo[0] = g2[i][0]; lo[1] = g2[i][1]; lo[2] = g2[i][2]; lo[3] = g2[i][3];
      hi[0] = g2[i][4]; hi[1] = g2[i][5]; hi[2] = g2[i][6]; hi[3] = g2[i][7];
      *reinterpret_cast<bf16x4*>(&sW2[buf][row * kW2Ld + w2_slot(8 * q)]) = lo;
      *reinterpret_cast<bf16x4*>(&sW2[buf][row * kW2Ld + w2_slot(8 * q + 4)]) = hi;
    }
    if (tid < 32) sB1[buf][tid] = gb;
  };

  gload(0);
  // ---- this lane's token row as X^T fragments: element j of k-step s = X[tok][16 s + 8 h2 + j] ----
  bf16x8 xf[KS];
  {
    const float* xr = X + (long)tokc * D + 8 * h2;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(xr + 16 * s);
      const float4 b = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
      xf[s][0] = (__bf16)a.x; xf[s][1] = (__bf16)a.y; xf[s][2] = (__bf16)a.z; xf[s][3] = (__bf16)a.w;
      xf[s][4] = (__bf16)b.x; xf[s][5] = (__bf16)b.y; xf[s][6] = (__bf16)b.z; xf[s][7] = (__bf16)b.w;
    }
  }
  sstore(0);
  __syncthreads();

  f32x16 o[OT];
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;

  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) gload(c + 1);
    // H^T = W1_c X^T: rows = hidden units (registers), cols = tokens (lanes)
    f32x16 hacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[r] = 0.f;
    const __bf16* w1 = &sW1[cur][col * W1LD + 8 * h2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      hacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w1 + 16 * s),
                                                     xf[s], hacc, 0, 0, 0);
    // + b1, SwooshL, bf16: the two k-step fragments of the second product
    bf16x8 pf[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int hrow = (r & 3) + 8 * (r >> 2) + 4 * h2;
      pf[r >> 3][r & 7] = (__bf16)swooshl_fast(hacc[r] + sB1[cur][hrow]);
    }
    // O^T += W2_c H^T: rows = output channels t*32 + col (A fragment from the permuted chunk)
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const __bf16* w2 = &sW2[cur][(t * 32 + col) * kW2Ld + 8 * h2];
      o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w2), pf[0], o[t], 0, 0, 0);
      o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w2 + 16), pf[1], o[t], 0, 0, 0);
    }
    if (c + 1 < nch) sstore(cur ^ 1);
    __syncthreads();
  }

  // ---- X[tok][d] += O^T + b2: lane's token, channels t*32 + 8 g + 4 h2 + (0..3) ----
  if (tok >= R) return;
  float* xr = X + (long)tok * D;
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = t * 32 + 8 * g + 4 * h2;
      const float4 bb = *reinterpret_cast<const float4*>(b2 + ch);
      float4 v = *reinterpret_cast<const float4*>(xr + ch);
      v.x += o[t][4 * g + 0] + bb.x;
      v.y += o[t][4 * g + 1] + bb.y;
      v.z += o[t][4 * g + 2] + bb.z;
      v.w += o[t][4 * g + 3] + bb.w;
      if (byp_orig != nullptr) {  // bypass_mid folded in (launch_bypass's formula)
        const float4 b0 = *reinterpret_cast<const float4*>(byp_orig + (long)tok * D + ch);
        const float4 k = *reinterpret_cast<const float4*>(byp_scale + ch);
        v.x = b0.x + (v.x - b0.x) * k.x;
        v.y = b0.y + (v.y - b0.y) * k.y;
        v.z = b0.z + (v.z - b0.z) * k.z;
        v.w = b0.w + (v.w - b0.w) * k.w;
      }
      *reinterpret_cast<float4*>(xr + ch) = v;
    }
}

// Wide model dims (256, 384, 512), where the one-wave-per-32-tokens design above runs out of
// registers: a block of 8 waves (two per SIMD, so one wave's loads hide behind the other's
// MFMAs) owns a 64-token tile held once in LDS as bf16, and per 128-unit hidden chunk
//   phase A  H^T = W1_c X^T     wave w computes hidden units 16 w .. 16 w + 15 for the four
//                               16-token tiles (v_mfma_f32_16x16x32_bf16; A = W1 rows from
//                               global/L2, B = X^T from LDS): each W1 fragment feeds 4 MFMAs
//   (+ b1, SwooshL, bf16 -> the chunk's H in LDS, [token][hidden])
//   phase B  O^T += W2_c H^T    wave w owns output channels [w D/8, (w + 1) D/8) for all 64
//                               tokens (A = W2 rows from global/L2, B = H^T from LDS)
// so the hidden activation never leaves the CU and each weight element is read once per
// block (256 B per hidden unit per 64 tokens).  Weight fragments are register-prefetched a
// phase ahead: the chunk's W2 fragments are issued before its phase A, the next chunk's W1
// fragments right after this chunk's phase A.  Two barriers per chunk around the H write.
// Epilogue as above: X += O^T + b2 (+ bypass_mid).
template <int D, bool EB = true>
__global__ __launch_bounds__(512, 1) void ffn_wide_kernel(float* __restrict__ X, int R, int F,
                                                          const __bf16* __restrict__ W1,
                                                          const float* __restrict__ b1,
                                                          const __bf16* __restrict__ W2,
                                                          const float* __restrict__ b2,
                                                          const float* __restrict__ byp_orig,
                                                          const float* __restrict__ byp_scale) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int TT = 64, HC = 128, NW = 8;
  // bf16 row strides of 16 (8 k + 2) bytes: the 16x16x32 operand reads (row = lane & 15,
  // 16-byte column chunk lane >> 4) then hit 16 distinct 16-byte bank slots in each of
  // ds_read_b128's four 16-lane groups (an odd multiple of 16 B suits 32x32 reads, not these)
  constexpr int XLD = D + 16, HLD = HC + 16;
  constexpr int KS = D / 32;                // phase-A k-steps (K = 32 per MFMA)
  constexpr int OW = D / NW, OT = OW / 16;  // output channels / 16-row tiles per wave
  __shared__ __attribute__((aligned(16))) __bf16 sX[TT * XLD];
  constexpr int NB = D >= 384 ? 2 : 1;  // H buffers (double-buffering measured slower at 256)
  __shared__ __attribute__((aligned(16))) __bf16 sH[NB][TT * HLD];
  __shared__ __attribute__((aligned(16))) float sB1[kMaxF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar branches
  const int r16 = lane & 15, g4 = lane >> 4;
  const long t0 = (long)blockIdx.x * TT;

  FFN_STAMP(0)
  // ---- X tile -> bf16 LDS (rows past R: a clamped duplicate, never written back) ----
  {
    constexpr int NE = TT * D / 4 / (64 * NW);
    float4 v[NE];
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
      const long r = t0 + row < R ? t0 + row : R - 1;
      v[i] = *reinterpret_cast<const float4*>(X + r * D + 4 * c4);
    }
#pragma unroll
    for (int i = 0; i < NE; ++i) {
      const int e = tid + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
      bf16x4 b;
      b[0] = (__bf16)v[i].x; b[1] = (__bf16)v[i].y; b[2] = (__bf16)v[i].z; b[3] = (__bf16)v[i].w;
      *reinterpret_cast<bf16x4*>(&sX[row * XLD + 4 * c4]) = b;
    }
  }

  f32x4 o[OT][4];
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) o[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = (F + HC - 1) / HC;
  // unconditional loads (a guarded load becomes a branch whose waits drain every load in
  // flight): W1 rows past F clamp to row F - 1, W2 columns past F clamp into the row; both
  // meet zero H (see below)
  // W1 / W2 in MFMA-fragment order (ffn_pack_weights): every fragment load is one
  // contiguous 1 KB wave read
  const int S2 = F / 32;  // k-steps of a W2 row group
  bf16x8 w1f[KS];
  auto load_w1 = [&](int c) {
    const int rg = min((c * HC) / 16 + wid, F / 16 - 1);
    const __bf16* p = W1 + ((long)rg * KS * 64 + lane) * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) w1f[s] = *reinterpret_cast<const bf16x8*>(p + s * 512);
  };
#ifndef ZASR_FFN_W2SETS
#define ZASR_FFN_W2SETS 2
#endif

  // W2SETS = 2: two W2 register sets; chunk c + 1's W2 goes out right after chunk c's H
  // barrier (with its W1), so it has chunk c's phase B AND chunk c + 1's phase A to land
  // instead of phase A alone.  W2SETS = 1: the single set reloaded after phase B.
  constexpr int W2S = ZASR_FFN_W2SETS;
  // Measured and dropped (profiles/r03/ffn_w2sets/): phase A token-sub-tile outer with each
  // sub-tile's SwooshL / H write interleaved (phase A 2200 -> 3800 cycles, 10-16 % slower);
  // a software-pipelined loop running chunk c + 1's phase A in the instruction stream of
  // chunk c's SwooshL / H write, with and without sched_group_barrier interleaving (the
  // SwooshL VALU stayed a ~2000-cycle block after the MFMAs; +-2 %, no gain).
  bf16x8 w2f[W2S][4][OT];
  auto load_w2 = [&](int c, auto set) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ks = min(c * (HC / 32) + s, S2 - 1);
#pragma unroll
      for (int t = 0; t < OT; ++t)
        w2f[S][s][t] = *reinterpret_cast<const bf16x8*>(W2 + (((long)(wid * OW / 16 + t) * S2 + ks) * 64 + lane) * 8);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, W2S - 1>;
  load_w1(0);
  load_w2(0, I0{});
  for (int e = tid; e < F; e += 64 * NW) sB1[e] = b1[e];
  lds_barrier();
  FFN_STAMP(1)
  auto chunk = [&](int c, auto set) {
    constexpr int S = decltype(set)::value;
    const int hid0 = c * HC + wid * 16;
    const bool hvalid = hid0 < F;  // F % 16 == 0: a wave's 16 units are all valid or none
    FFN_STAMP(2 + 4 * c)
    __bf16* sHc = sH[NB == 2 ? (c & 1) : 0];
    f32x4 ha[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) ha[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(&sX[(16 * u + r16) * XLD + 32 * s + 8 * g4]);
        ha[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[s], xb, ha[u], 0, 0, 0);
      }
    }
    FFN_STAMP(3 + 4 * c)
    // two buffers: H goes to buffer c & 1; every wave finished reading it (chunk c - 2's
    // phase B) before it passed chunk c - 1's barrier, which precedes this write.  One
    // buffer: a barrier first, so the previous chunk's phase B is done everywhere
    if constexpr (NB == 1) lds_barrier();
    FFN_STAMP(4 + 4 * c)
    if (hvalid) {
      const float4 bb = *reinterpret_cast<const float4*>(&sB1[hid0 + 4 * g4]);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        bf16x4 p;
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = (__bf16)swooshl_fast(ha[u][q] + bv[q]);
        *reinterpret_cast<bf16x4*>(&sHc[(16 * u + r16) * HLD + wid * 16 + 4 * g4]) = p;
      }
    } else {  // hidden units past F (tail chunk): zero H columns
      const bf16x4 z = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) *reinterpret_cast<bf16x4*>(&sHc[(16 * u + r16) * HLD + wid * 16 + 4 * g4]) = z;
    }
    lds_barrier();
    FFN_STAMP(5 + 4 * c)
    // in-order vmcnt: the next chunk's W1 (needed first) is issued before its W2
    load_w1(min(c + 1, nch - 1));  // unconditional: a branch here costs exact vmcnt tracking
    if constexpr (W2S == 2) load_w2(min(c + 1, nch - 1), std::integral_constant<int, 1 - S>{});
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 hf[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) hf[u] = *reinterpret_cast<const bf16x8*>(&sHc[(16 * u + r16) * HLD + 32 * s + 8 * g4]);
#pragma unroll
      for (int t = 0; t < OT; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) o[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[S][s][t], hf[u], o[t][u], 0, 0, 0);
    }
    if constexpr (W2S == 1) load_w2(min(c + 1, nch - 1), I0{});
  };
  for (int c = 0; c < nch; c += W2S) {
    chunk(c, I0{});
    if constexpr (W2S == 2) {
      if (c + 1 < nch) chunk(c + 1, I1{});
    }
  }

  // ---- X[tok][ch] += O^T + b2 (+ bypass_mid): lane's token, 4 consecutive channels ----
  if constexpr (EB) {
    // the residual (and bypass) pieces of two row groups loaded together, rows past R clamped
    // (loaded, never stored): two memory round trips instead of one per row group
    float4 bv[OT], kv[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int ch = wid * OW + 16 * t + 4 * g4;
      bv[t] = *reinterpret_cast<const float4*>(b2 + ch);
      if (byp_orig != nullptr) kv[t] = *reinterpret_cast<const float4*>(byp_scale + ch);
    }
#pragma unroll
    for (int u0 = 0; u0 < 4; u0 += 2) {
    float4 xv[2][OT], b0v[2][OT];
#pragma unroll
    for (int du = 0; du < 2; ++du) {
      const long tok = min(t0 + 16 * (u0 + du) + r16, (long)R - 1);
#pragma unroll
      for (int t = 0; t < OT; ++t) {
        const int ch = wid * OW + 16 * t + 4 * g4;
        xv[du][t] = *reinterpret_cast<const float4*>(X + tok * D + ch);
        if (byp_orig != nullptr) b0v[du][t] = *reinterpret_cast<const float4*>(byp_orig + tok * D + ch);
      }
    }
#pragma unroll
    for (int du = 0; du < 2; ++du) {
      const int u = u0 + du;
      const long tok = t0 + 16 * u + r16;
      if (tok >= R) continue;
      float* xr = X + tok * D;
#pragma unroll
      for (int t = 0; t < OT; ++t) {
        const int ch = wid * OW + 16 * t + 4 * g4;
        float4 v = xv[du][t];
        v.x += o[t][u][0] + bv[t].x;
        v.y += o[t][u][1] + bv[t].y;
        v.z += o[t][u][2] + bv[t].z;
        v.w += o[t][u][3] + bv[t].w;
        if (byp_orig != nullptr) {
          const float4 b0 = b0v[du][t], k = kv[t];
          v.x = b0.x + (v.x - b0.x) * k.x;
          v.y = b0.y + (v.y - b0.y) * k.y;
          v.z = b0.z + (v.z - b0.z) * k.z;
          v.w = b0.w + (v.w - b0.w) * k.w;
        }
        *reinterpret_cast<float4*>(xr + ch) = v;
      }
    }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long tok = t0 + 16 * u + r16;
    if (tok >= R) continue;
    float* xr = X + tok * D;
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int ch = wid * OW + 16 * t + 4 * g4;
      const float4 bv = *reinterpret_cast<const float4*>(b2 + ch);
      float4 v = *reinterpret_cast<const float4*>(xr + ch);
      v.x += o[t][u][0] + bv.x;
      v.y += o[t][u][1] + bv.y;
      v.z += o[t][u][2] + bv.z;
      v.w += o[t][u][3] + bv.w;
      if (byp_orig != nullptr) {
        const float4 b0 = *reinterpret_cast<const float4*>(byp_orig + tok * D + ch);
        const float4 k = *reinterpret_cast<const float4*>(byp_scale + ch);
        v.x = b0.x + (v.x - b0.x) * k.x;
        v.y = b0.y + (v.y - b0.y) * k.y;
        v.z = b0.z + (v.z - b0.z) * k.z;
        v.w = b0.w + (v.w - b0.w) * k.w;
      }
      *reinterpret_cast<float4*>(xr + ch) = v;
    }
  }
}

// ffn_wide_kernel over a per-CU share of the rows ("rows" form, d = 384): one block per CU
// walks rpb rows (a multiple of 16) in 64-token tiles and a 16-48-token tail tile.  One block
// per 64-token tile ran d = 384's 773 tiles in 4 rounds of the 256 CUs for 3.02 rounds of
// work: the rows form measured 1.08-1.10x at F = 768 / 1024 / 1280, bit-identical
// (tools/ffnw_lab.hip, profiles/r06/ffn_rows/).  Not at d = 256 (0.82-0.87x: one block per
// tile runs two blocks per CU whose X staging and epilogues overlap each other's chunks; the
// rows form at two blocks per CU spills) nor d = 512 (0.95x, spills).
template <int D, bool EB>
__global__ __launch_bounds__(512, 2) void ffn_rows_kernel(float* __restrict__ X, int R, int F,
                                                          const __bf16* W1,
                                                          const float* __restrict__ b1,
                                                          const __bf16* W2,
                                                          const float* __restrict__ b2,
                                                          const float* __restrict__ byp_orig,
                                                          const float* __restrict__ byp_scale,
                                                          int rpb) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int TUM = 4, HC = 128, NW = 8;
  constexpr int XLD = D + 16, HLD = HC + 16;  // as ffn_wide_kernel
  constexpr int KS = D / 32;
  constexpr int OW = D / NW, OT = OW / 16;
  __shared__ __attribute__((aligned(16))) __bf16 sX[16 * TUM * XLD];
  constexpr int NB = D >= 384 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) __bf16 sH[NB][16 * TUM * HLD];
  __shared__ __attribute__((aligned(16))) float sB1[kMaxF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const long r0 = (long)blockIdx.x * rpb;
  const long r1 = r0 + rpb < R ? r0 + rpb : R;
  const int nch = (F + HC - 1) / HC;
  const int S2 = F / 32;
  bf16x8 w1f[KS];
  auto load_w1 = [&](int c) {
    const int rg = min((c * HC) / 16 + wid, F / 16 - 1);
    const __bf16* p = W1 + ((long)rg * KS * 64 + lane) * 8;
#pragma unroll
    for (int s = 0; s < KS; ++s) w1f[s] = *reinterpret_cast<const bf16x8*>(p + s * 512);
  };
  constexpr int W2S = ZASR_FFN_W2SETS;
  bf16x8 w2f[W2S][4][OT];
  auto load_w2 = [&](int c, auto set) {
    constexpr int S = decltype(set)::value;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int ks = min(c * (HC / 32) + s, S2 - 1);
#pragma unroll
      for (int t = 0; t < OT; ++t)
        w2f[S][s][t] = *reinterpret_cast<const bf16x8*>(W2 + (((long)(wid * OW / 16 + t) * S2 + ks) * 64 + lane) * 8);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, W2S - 1>;
  for (int e = tid; e < F; e += 64 * NW) sB1[e] = b1[e];  // published by the first X barrier

  auto tile = [&](auto tu_c, const long t0) __attribute__((always_inline)) {
    constexpr int TU = decltype(tu_c)::value, TT = 16 * TU;
    // the X tile's element indices and addresses from a per-tile copy of tid: hoisted out of
    // the tile loop they stay live through it (24+ VGPRs at d = 384: spills)
    int tix = tid;
    asm volatile("" : "+v"(tix));
    // ---- X tile -> bf16 LDS (rows past R: a clamped duplicate, never written back); every
    // wave read the previous tile's sX (its last phase A) before the last H barrier ----
    {
      static_assert(TT * D / 4 % (64 * NW) == 0, "X tile staging");
      constexpr int NE = TT * D / 4 / (64 * NW);
      float4 v[NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = tix + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
        const long r = t0 + row < R ? t0 + row : R - 1;
        v[i] = *reinterpret_cast<const float4*>(X + r * D + 4 * c4);
      }
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = tix + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
        bf16x4 b;
        b[0] = (__bf16)v[i].x; b[1] = (__bf16)v[i].y; b[2] = (__bf16)v[i].z; b[3] = (__bf16)v[i].w;
        *reinterpret_cast<bf16x4*>(&sX[row * XLD + 4 * c4]) = b;
      }
    }
    // the first chunk's weights, behind the X tile (a prefetch from the previous tile's last
    // chunk, or ahead of the X loads, holds the weight registers live through the epilogue /
    // the X conversion: 256 VGPRs and scratch; W1 / W2 are not __restrict__, whose invariant
    // loads the compiler hoists out of the tile loop for the same effect)
    load_w1(0);
    load_w2(0, I0{});
    lds_barrier();  // (also: every wave is done with the previous tile's H buffers)

    f32x4 o[OT][TU];
#pragma unroll
    for (int t = 0; t < OT; ++t)
#pragma unroll
      for (int u = 0; u < TU; ++u) o[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto chunk = [&](int c, auto set) __attribute__((always_inline)) {
      constexpr int S = decltype(set)::value;
      const int hid0 = c * HC + wid * 16;
      const bool hvalid = hid0 < F;
      __bf16* sHc = sH[NB == 2 ? (c & 1) : 0];
      f32x4 ha[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) ha[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const bf16x8 xb = *reinterpret_cast<const bf16x8*>(&sX[(16 * u + r16) * XLD + 32 * s + 8 * g4]);
          ha[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1f[s], xb, ha[u], 0, 0, 0);
        }
      }
      if constexpr (NB == 1) lds_barrier();
      if (hvalid) {
        const float4 bb = *reinterpret_cast<const float4*>(&sB1[hid0 + 4 * g4]);
        const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          bf16x4 p;
#pragma unroll
          for (int q = 0; q < 4; ++q) p[q] = (__bf16)swooshl_fast(ha[u][q] + bv[q]);
          *reinterpret_cast<bf16x4*>(&sHc[(16 * u + r16) * HLD + wid * 16 + 4 * g4]) = p;
        }
      } else {
        const bf16x4 z = {(__bf16)0.f, (__bf16)0.f, (__bf16)0.f, (__bf16)0.f};
#pragma unroll
        for (int u = 0; u < TU; ++u) *reinterpret_cast<bf16x4*>(&sHc[(16 * u + r16) * HLD + wid * 16 + 4 * g4]) = z;
      }
      lds_barrier();
      // the next chunk's weights (unconditional: the last chunk's re-load is dead code)
      const int cn = min(c + 1, nch - 1);
      load_w1(cn);
      if constexpr (W2S == 2) load_w2(cn, std::integral_constant<int, 1 - S>{});
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 hf[TU];
#pragma unroll
        for (int u = 0; u < TU; ++u) hf[u] = *reinterpret_cast<const bf16x8*>(&sHc[(16 * u + r16) * HLD + 32 * s + 8 * g4]);
#pragma unroll
        for (int t = 0; t < OT; ++t)
#pragma unroll
          for (int u = 0; u < TU; ++u) o[t][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2f[S][s][t], hf[u], o[t][u], 0, 0, 0);
      }
      if constexpr (W2S == 1) load_w2(cn, I0{});
    };
    for (int c = 0; c < nch; c += W2S) {
      chunk(c, I0{});
      if constexpr (W2S == 2) {
        if (c + 1 < nch) chunk(c + 1, I1{});
      }
    }

    // ---- X[tok][ch] += O^T + b2 (+ bypass_mid): lane's token, 4 consecutive channels ----
    int g4e = g4;  // (per tile, as tix: the epilogue's b2 / scale loads and addresses)
    asm volatile("" : "+v"(g4e));
    float4 bv[OT], kv[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int ch = wid * OW + 16 * t + 4 * g4e;
      bv[t] = *reinterpret_cast<const float4*>(b2 + ch);
      if (byp_orig != nullptr) kv[t] = *reinterpret_cast<const float4*>(byp_scale + ch);
    }
    // EB: the residual (and bypass) pieces of two row groups loaded together
    constexpr int UB = EB ? 2 : 1;
#pragma unroll
    for (int u0 = 0; u0 < TU; u0 += UB) {
      float4 xv[UB][OT], b0v[UB][OT];
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        if (u0 + du >= TU) break;
        const long tok = min(t0 + 16 * (u0 + du) + r16, (long)R - 1);
#pragma unroll
        for (int t = 0; t < OT; ++t) {
          const int ch = wid * OW + 16 * t + 4 * g4e;
          xv[du][t] = *reinterpret_cast<const float4*>(X + tok * D + ch);
          if (byp_orig != nullptr) b0v[du][t] = *reinterpret_cast<const float4*>(byp_orig + tok * D + ch);
        }
      }
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        const int u = u0 + du;
        if (u >= TU) break;
        const long tok = t0 + 16 * u + r16;
        if (tok >= r1) continue;
        float* xr = X + tok * D;
#pragma unroll
        for (int t = 0; t < OT; ++t) {
          const int ch = wid * OW + 16 * t + 4 * g4e;
          float4 v = xv[du][t];
          v.x += o[t][u][0] + bv[t].x;
          v.y += o[t][u][1] + bv[t].y;
          v.z += o[t][u][2] + bv[t].z;
          v.w += o[t][u][3] + bv[t].w;
          if (byp_orig != nullptr) {
            const float4 b0 = b0v[du][t], k = kv[t];
            v.x = b0.x + (v.x - b0.x) * k.x;
            v.y = b0.y + (v.y - b0.y) * k.y;
            v.z = b0.z + (v.z - b0.z) * k.z;
            v.w = b0.w + (v.w - b0.w) * k.w;
          }
          *reinterpret_cast<float4*>(xr + ch) = v;
        }
      }
    }
  };

  using TM = std::integral_constant<int, TUM>;
  long t0 = r0;
  for (; t0 + 16 * TUM <= r1; t0 += 16 * TUM) tile(TM{}, t0);
  // 0-3 row groups left (rpb is a multiple of 16), up to 4 in the last block (R need not be)
  const int tail = (int)((r1 - t0 + 15) / 16);
  if (tail == 1) tile(std::integral_constant<int, 1>{}, t0);
  if (tail == 2) tile(std::integral_constant<int, 2>{}, t0);
  if (tail == 3) tile(std::integral_constant<int, 3>{}, t0);
  if (tail == 4) tile(TM{}, t0);
}

// ---- f16x3 wide FFN (the token-exact mode) ----
// The same FeedforwardModule at f32 quality: every product on fp16 MFMAs over the two pieces
// x = hi + lo 2^-11 (gemm_dev.h split_h8), here in the one-accumulator form -- the weight's hi
// piece scaled by 2^11 in registers (v_pk_mul_f16, exact for |w| < 32: ffn_h3_weights_ok),
// so the three products w_lo x_hi + w_hi x_lo + (w_hi 2^11) x_hi land on one 2^11-scaled
// accumulator (one register set per output fragment, as in the bf16 kernel).  The unfused
// f16x3 path writes the f32 hidden activation to HBM and reads it back (R F 8 bytes per FFN);
// here it stays on chip as fp16 pieces.  Structure of ffn_wide_kernel: 8 waves, one block per
// CU, a TT-token tile held once in LDS (two fp16 piece images, split once per block), 128
// hidden units per chunk:
//   phase A  H^T = W1_c X^T   wave w: hidden units 16 w .. 16 w + 15 x TT tokens
//                             (v_mfma_f32_16x16x32_f16; A = W1 pieces from L2, B = X pieces
//                             from LDS)
//   + b1, SwooshL, split -> the chunk's H pieces in LDS
//   phase B  O^T += W2_c H^T  wave w: output channels [w D/8, (w + 1) D/8) x TT tokens
// Weight fragments stream through small register rings (too many pieces to hold a chunk's
// set): W1 P1 k-steps ahead within phase A (the next chunk's first P1 issued in phase B), W2
// two k-steps ahead (the chunk's first two issued at the top of its phase A).
// W1 / W2 pieces: ffn_pack_host per piece, piece 1 at + F D elements.
namespace {
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr float kF16Lo = 2048.f, kF16LoInv = 1.f / 2048.f;  // gemm_dev.h's piece scale

// SwooshL of the 2^11-scaled accumulator as its two fp16 pieces (hi, lo 2^11), in 2^11 units
// throughout: ys = acc + 2^11 (b1 - 4) = 2^11 y with y = x - 4 (bs = that bias), so
//   2^11 SwooshL(x) = max(ys, 0) + 2^11 ln2 log2(1 + 2^(-|ys| log2(e) 2^-11)) - 0.08 ys - 2^11 0.355
// (softplus_fast's form), hi = fp16(r 2^-11), lo = fp16(r - 2^11 hi) by v_fma_mix (the fp16
// operand widened inside the instruction; the compiler does not form it from C): ~9 VALU and
// 2 transcendentals a value where scaling, shifting, widening and subtracting took ~12
__device__ __forceinline__ void swooshl_pieces2(float a0, float a1, float bs0, float bs1,
                                                _Float16& h0, _Float16& h1, _Float16& l0,
                                                _Float16& l1) {
  constexpr float kL = -1.4426950408889634f / 2048.f, kLn = 0.6931471805599453f * 2048.f;
  constexpr float kC = -0.355f * 2048.f;
  float r[2];
  const float ys[2] = {a0 + bs0, a1 + bs1};
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const float l = __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(fabsf(ys[q]) * kL));
    r[q] = fmaf(ys[q], -0.08f, fmaf(l, kLn, fmaxf(ys[q], 0.f))) + kC;
  }
  typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
  const f16x2_t hh = {(_Float16)(r[0] * (1.f / 2048.f)), (_Float16)(r[1] * (1.f / 2048.f))};
  const unsigned hu = __builtin_bit_cast(unsigned, hh);
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, %1, %4, %2 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %0, %1, %4, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(lo) : "v"(hu), "v"(r[0]), "v"(r[1]), "v"(-2048.f));
  const f16x2_t ll = __builtin_bit_cast(f16x2_t, lo);
  h0 = hh[0];
  h1 = hh[1];
  l0 = ll[0];
  l1 = ll[1];
}

// acc (2^11 scale) += w_lo x_hi + w_hi x_lo + w_s x_hi, w_s = w_hi 2^11; smallest terms first
__device__ __forceinline__ void mfma16_h3(f32x4v& acc, const f16x8& wh, const f16x8& wl,
                                          const f16x8& ws, const f16x8& xh, const f16x8& xl) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ws, xh, acc, 0, 0, 0);
}
}  // namespace

// SB (split barrier; NB == 1): the chunk's two block barriers become LDS counters per half of
// the hidden chunk.  Waves 0 .. NW/2 - 1 own units [0, HC/2), the others [HC/2, HC); phase B's
// first HC/64 k-steps read only the low half.  A wave writes its half of H(c) once every wave
// has finished reading that half of H(c - 1), announces it, waits for the LOW half to be
// complete, runs the low k-steps, announces them read, and waits for the high half only
// before its high k-steps -- so the waves that finish phase A first (waves 0 .. 3 issue ahead
// of their SIMD partners) run their low phase-B MFMAs while the partners are still in
// SwooshL, instead of idling at a block barrier (per-wave stamps: profiles/r06/ffn_pp/).
// Same products in the same order: bit-identical to the barrier form.
template <int D, int TUM, int NB, int NW, bool SB = false, bool EB = false>
__global__ __launch_bounds__(64 * NW, 8 / NW) void ffn_wide_h3_kernel(float* __restrict__ X, int R, int F,
                                                             const __bf16* __restrict__ W1,
                                                             const float* __restrict__ b1,
                                                             const __bf16* __restrict__ W2,
                                                             const float* __restrict__ b2,
                                                             const float* __restrict__ byp_orig,
                                                             const float* __restrict__ byp_scale,
                                                             int rpb, const float* __restrict__ Y) {
  constexpr int HC = 16 * NW, TTM = 16 * TUM;  // NW waves: 8 (one block per CU), 4 (two)
  constexpr int XLD = D + 16, HLD = HC + 16;  // 16 (8 k + 2)-byte rows, as ffn_wide_kernel
  constexpr int KS = D / 32;
  constexpr int OW = D / NW, OT = OW / 16;
  constexpr int P1 = KS < 3 ? KS : 3;
  static_assert(OW % 16 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) _Float16 sX[2][TTM * XLD];
  __shared__ __attribute__((aligned(16))) _Float16 sH[NB][2][TTM * HLD];
  // SB: waves that wrote H low / high, waves done reading H low / high (cumulative counts)
  __shared__ int sFlag[4];
  static_assert(!SB || NB == 1, "split barriers: one H buffer");

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  if (SB && tid < 4) sFlag[tid] = 0;  // visible after the first tile's X barrier
  const bool lo_half = wid < NW / 2;
  int gc = 0;  // chunks done by this block (all tiles): the counters' targets
  // this block's rows [r0, r1): rpb (a multiple of 16) per block, one block per CU, so every
  // CU gets the same share instead of a last round of a few TTM-row tiles
  const long r0 = (long)blockIdx.x * rpb;
  const long r1 = r0 + rpb < R ? r0 + rpb : R;
  const long PC = (long)F * D;  // elements per piece image (W1 and W2 alike)
  const int S2 = F / 32;
  const int nch = (F + HC - 1) / HC;
  const f16x8 kS = {(_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f,
                    (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f};

  // ---- weight rings (unconditional, clamped loads: rows / k-steps past F meet zero H) ----
  f16x8 w1r[P1][2];
  // fragments by buffer loads: the fragment's byte offset is wave-uniform (an SGPR) and the
  // lane's 16 bytes a constant VGPR -- no 64-bit address arithmetic per load in the loops
  const int voff = lane * 16, pcb = (int)(PC * 2);
  const __amdgpu_buffer_rsrc_t rs1 = wave_rsrc(W1, 4 * PC), rs2 = wave_rsrc(W2, 4 * PC);
  auto load_w1 = [&](int c, int s, int slot) {
    const int rg = min((c * HC) / 16 + wid, F / 16 - 1);
    const int so = (rg * KS + s) * 1024;
    w1r[slot][0] = buf_load16<f16x8>(rs1, voff, so);
    w1r[slot][1] = buf_load16<f16x8>(rs1, voff, so + pcb);
  };
  f16x8 w2r[2][OT][2];
  auto load_w2 = [&](int c, int s, int slot) {
    const int ks = min(c * (HC / 32) + s, S2 - 1);
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int so = ((wid * OT + t) * S2 + ks) * 1024;
      w2r[slot][t][0] = buf_load16<f16x8>(rs2, voff, so);
      w2r[slot][t][1] = buf_load16<f16x8>(rs2, voff, so + pcb);
    }
  };
  FFN_STAMP(0)
#pragma unroll
  for (int s = 0; s < P1; ++s) load_w1(0, s, s);

  // one tile of TU x 16 rows from t0 (the block's whole tiles at TUM, its last one at what is
  // left); the weight rings run on across tiles (the last chunk prefetches chunk 0)
#ifdef ZASR_FFN_STAMPS
  int kt = 0;  // development: per-tile stamps at 1000 + 100 kt (tools/ffnh3_lab.hip)
#define FFN_TSTAMP(i) FFN_STAMP(1000 + 100 * (kt < 30 ? kt : 30) + (i))
  // every wave of block 0, tile 1: 4000 + 100 wave + 4 c + phase
#define FFN_WSTAMP(i) \
  if (blockIdx.x == 0 && lane == 0 && kt == 1) g_ffn_stamps[4000 + 100 * wid + (i)] = clock64();
#else
#define FFN_TSTAMP(i)
#define FFN_WSTAMP(i)
#endif
  auto tile = [&](auto tu_c, const long t0) {
  constexpr int TU = decltype(tu_c)::value, TT = 16 * TU;
  FFN_TSTAMP(0)
  // ---- X tile -> two fp16 piece images (rows past R: a clamped duplicate, never written) ----
  {
    constexpr int NE = TT * D / 4 / (64 * NW);
    static_assert(NE * 64 * NW * 4 == TT * D, "X tile split");
    constexpr int NH = NE % 2 == 0 ? NE / 2 : NE;  // in two halves (registers)
#pragma unroll
    for (int i0 = 0; i0 < NE; i0 += NH) {
    float4 v[NH];
#pragma unroll
    for (int i = i0; i < i0 + NH; ++i) {
      const int e = tid + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
      const long r = t0 + row < R ? t0 + row : R - 1;
      v[i - i0] = *reinterpret_cast<const float4*>(Y + r * D + 4 * c4);
    }
#pragma unroll
    for (int i = i0; i < i0 + NH; ++i) {
      const int e = tid + 64 * NW * i, row = e / (D / 4), c4 = e - row * (D / 4);
      const float x4[4] = {v[i - i0].x, v[i - i0].y, v[i - i0].z, v[i - i0].w};
      f16x4 hh, ll;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        hh[q] = (_Float16)x4[q];
        ll[q] = (_Float16)((x4[q] - (float)hh[q]) * kF16Lo);
      }
      *reinterpret_cast<f16x4*>(&sX[0][row * XLD + 4 * c4]) = hh;
      *reinterpret_cast<f16x4*>(&sX[1][row * XLD + 4 * c4]) = ll;
    }
    }
  }
  lds_barrier();
  FFN_STAMP(1)
  FFN_TSTAMP(1)

  f32x4v o[OT][TU];
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int u = 0; u < TU; ++u) o[t][u] = f32x4v{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nch; ++c) {
    const int hid0 = c * HC + wid * 16;
    const bool hvalid = hid0 < F;  // F % 16 == 0: a wave's 16 units are all valid or none
    // this chunk's first two W2 k-steps (their ring slots were consumed by the last phase B)
    // b1 of the wave's 16 units (4 per lane group g4): a volatile load keeps its place ahead
    // of phase A (a plain one is sunk next to its use, behind a full wait)
    const f32x4v bb = *reinterpret_cast<const volatile f32x4v*>(b1 + min(hid0, F - 16) + 4 * g4);
    load_w2(c, 0, 0);
    load_w2(c, 1, 1);
    // loads stay where they are issued (the scheduler would sink them next to their use)
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase A: step s + 1's X fragments are read before step s's MFMAs ----
    f32x4v ha[TU];
#pragma unroll
    for (int u = 0; u < TU; ++u) ha[u] = f32x4v{0.f, 0.f, 0.f, 0.f};
    f16x8 xf[2][TU][2];
    auto read_x = [&](int s, int buf) {
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int xo = (16 * u + r16) * XLD + 32 * s + 8 * g4;
        xf[buf][u][0] = *reinterpret_cast<const f16x8*>(&sX[0][xo]);
        xf[buf][u][1] = *reinterpret_cast<const f16x8*>(&sX[1][xo]);
      }
    };
    FFN_STAMP(8 + 4 * c)
    FFN_TSTAMP(2 + 4 * (c & 15))
    FFN_WSTAMP(4 * (c & 15) + 0)
    read_x(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int slot = s % P1;
      if (s + 1 < KS) read_x(s + 1, (s + 1) & 1);
      const f16x8 wh = w1r[slot][0], wl = w1r[slot][1];
      const f16x8 ws = wh * kS;
#pragma unroll
      for (int u = 0; u < TU; ++u) mfma16_h3(ha[u], wh, wl, ws, xf[s & 1][u][0], xf[s & 1][u][1]);
      if (s + P1 < KS) load_w1(c, s + P1, slot);
      __builtin_amdgcn_sched_barrier(0);
    }
    FFN_STAMP(9 + 4 * c)
    FFN_TSTAMP(3 + 4 * (c & 15))
    FFN_WSTAMP(4 * (c & 15) + 1)
    // ---- + b1, SwooshL, split -> H pieces ----
    _Float16* sH0 = sH[NB == 2 ? (c & 1) : 0][0];
    _Float16* sH1 = sH[NB == 2 ? (c & 1) : 0][1];
    if constexpr (SB) {  // every wave has read this wave's half of H(c - 1)
      if (gc > 0) lds_wait_ge(&sFlag[lo_half ? 2 : 3], NW * gc);
    } else if constexpr (NB == 1) {
      lds_barrier();  // the previous chunk's phase B is done with sH
    }
    {
      // hidden units past F: zero H, the pieces masked (no branch: its waits would drain the
      // weight loads in flight)
      const float bs[4] = {2048.f * (bb[0] - 4.f), 2048.f * (bb[1] - 4.f), 2048.f * (bb[2] - 4.f),
                           2048.f * (bb[3] - 4.f)};
      const f16x4 hmk = hvalid ? f16x4{(_Float16)1.f, (_Float16)1.f, (_Float16)1.f, (_Float16)1.f}
                               : f16x4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        _Float16 h4[4], l4[4];
        swooshl_pieces2(ha[u][0], ha[u][1], bs[0], bs[1], h4[0], h4[1], l4[0], l4[1]);
        swooshl_pieces2(ha[u][2], ha[u][3], bs[2], bs[3], h4[2], h4[3], l4[2], l4[3]);
        const f16x4 hh = f16x4{h4[0], h4[1], h4[2], h4[3]} * hmk;
        const f16x4 ll = f16x4{l4[0], l4[1], l4[2], l4[3]} * hmk;
        const int ho = (16 * u + r16) * HLD + wid * 16 + 4 * g4;
        *reinterpret_cast<f16x4*>(&sH0[ho]) = hh;
        *reinterpret_cast<f16x4*>(&sH1[ho]) = ll;
      }
    }
    if constexpr (SB) {
      lds_signal(&sFlag[lo_half ? 0 : 1], lane);
      lds_wait_ge(&sFlag[0], (NW / 2) * (gc + 1));  // the low half of H(c) is complete
    } else {
      lds_barrier();
    }
    FFN_STAMP(10 + 4 * c)
    FFN_TSTAMP(4 + 4 * (c & 15))
    FFN_WSTAMP(4 * (c & 15) + 2)
    // ---- phase B: step s + 1's H fragments are read before step s's MFMAs ----
    f16x8 hf[2][TU][2];
    auto read_h = [&](int s, int buf) {
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int ho = (16 * u + r16) * HLD + 32 * s + 8 * g4;
        hf[buf][u][0] = *reinterpret_cast<const f16x8*>(&sH0[ho]);
        hf[buf][u][1] = *reinterpret_cast<const f16x8*>(&sH1[ho]);
      }
    };
    constexpr int SL = HC / 64;  // the first k-step over the high half of the chunk
    read_h(0, 0);
#pragma unroll
    for (int s = 0; s < HC / 32; ++s) {
      if (s + 1 < HC / 32 && !(SB && s + 1 == SL)) read_h(s + 1, (s + 1) & 1);
#pragma unroll
      for (int t = 0; t < OT; ++t) {
        const f16x8 wh = w2r[s & 1][t][0], wl = w2r[s & 1][t][1];
        const f16x8 ws = wh * kS;
#pragma unroll
        for (int u = 0; u < TU; ++u) mfma16_h3(o[t][u], wh, wl, ws, hf[s & 1][u][0], hf[s & 1][u][1]);
      }
      if (s + 2 < HC / 32) load_w2(c, s + 2, s & 1);
      if (s == 1) {  // the next chunk's first W1 k-steps (in-order vmcnt: after W2 step 3)
        const int cn = c + 1 < nch ? c + 1 : 0;  // (the next tile's first chunk)
#pragma unroll
        for (int q = 0; q < P1; ++q) load_w1(cn, q, q);
      }
      if constexpr (SB) {
        if (s == SL - 1) {  // low half read; the high half once its writers are done
          lds_signal(&sFlag[2], lane);
          lds_wait_ge(&sFlag[1], (NW / 2) * (gc + 1));
          read_h(SL, SL & 1);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (SB) lds_signal(&sFlag[3], lane);
    ++gc;
    FFN_STAMP(11 + 4 * c)
    FFN_TSTAMP(5 + 4 * (c & 15))
    FFN_WSTAMP(4 * (c & 15) + 3)
  }

  // ---- X[tok][ch] += O^T 2^-11 + b2 (+ bypass_mid) ----
  if constexpr (EB) {
    // the residual (and bypass) rows of up to two 16-row groups loaded together, rows past r1
    // clamped (loaded, never stored): one memory round trip per group pair instead of one
    // per (group, channel tile) behind each row guard (the tile's epilogue was ~9 % of it)
    float4 bv[OT], kv[OT];
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int ch = wid * OW + 16 * t + 4 * g4;
      bv[t] = *reinterpret_cast<const float4*>(b2 + ch);
      if (byp_orig != nullptr) kv[t] = *reinterpret_cast<const float4*>(byp_scale + ch);
    }
#pragma unroll
    for (int u0 = 0; u0 < TU; u0 += 2) {
      constexpr int UB = TU >= 2 ? 2 : 1;
      float4 xv[UB][OT], b0v[UB][OT];
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        if (u0 + du >= TU) break;
        const long tok = min(t0 + 16 * (u0 + du) + r16, r1 - 1);
#pragma unroll
        for (int t = 0; t < OT; ++t) {
          const int ch = wid * OW + 16 * t + 4 * g4;
          xv[du][t] = *reinterpret_cast<const float4*>(X + tok * D + ch);
          if (byp_orig != nullptr) b0v[du][t] = *reinterpret_cast<const float4*>(byp_orig + tok * D + ch);
        }
      }
#pragma unroll
      for (int du = 0; du < UB; ++du) {
        const int u = u0 + du;
        if (u >= TU) break;
        const long tok = t0 + 16 * u + r16;
        if (tok >= r1) continue;
        float* xr = X + tok * D;
#pragma unroll
        for (int t = 0; t < OT; ++t) {
          const int ch = wid * OW + 16 * t + 4 * g4;
          float4 v = xv[du][t];
          v.x += o[t][u][0] * kF16LoInv + bv[t].x;
          v.y += o[t][u][1] * kF16LoInv + bv[t].y;
          v.z += o[t][u][2] * kF16LoInv + bv[t].z;
          v.w += o[t][u][3] * kF16LoInv + bv[t].w;
          if (byp_orig != nullptr) {
            const float4 b0 = b0v[du][t], k = kv[t];
            v.x = b0.x + (v.x - b0.x) * k.x;
            v.y = b0.y + (v.y - b0.y) * k.y;
            v.z = b0.z + (v.z - b0.z) * k.z;
            v.w = b0.w + (v.w - b0.w) * k.w;
          }
          *reinterpret_cast<float4*>(xr + ch) = v;
        }
      }
    }
  } else {
#pragma unroll
  for (int u = 0; u < TU; ++u) {
    const long tok = t0 + 16 * u + r16;
    if (tok >= r1) continue;
    float* xr = X + tok * D;
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const int ch = wid * OW + 16 * t + 4 * g4;
      const float4 bv = *reinterpret_cast<const float4*>(b2 + ch);
      float4 v = *reinterpret_cast<const float4*>(xr + ch);
      v.x += o[t][u][0] * kF16LoInv + bv.x;
      v.y += o[t][u][1] * kF16LoInv + bv.y;
      v.z += o[t][u][2] * kF16LoInv + bv.z;
      v.w += o[t][u][3] * kF16LoInv + bv.w;
      if (byp_orig != nullptr) {
        const float4 b0 = *reinterpret_cast<const float4*>(byp_orig + tok * D + ch);
        const float4 k = *reinterpret_cast<const float4*>(byp_scale + ch);
        v.x = b0.x + (v.x - b0.x) * k.x;
        v.y = b0.y + (v.y - b0.y) * k.y;
        v.z = b0.z + (v.z - b0.z) * k.z;
        v.w = b0.w + (v.w - b0.w) * k.w;
      }
      *reinterpret_cast<float4*>(xr + ch) = v;
    }
  }
  }
  FFN_TSTAMP(90)
#ifdef ZASR_FFN_STAMPS
  ++kt;
#endif
  };  // tile

  using T1 = std::integral_constant<int, 1>;
  using T2 = std::integral_constant<int, 2>;
  using T3 = std::integral_constant<int, 3>;
  using TM = std::integral_constant<int, TUM>;
  long t0 = r0;
  for (; t0 + TTM <= r1; t0 += TTM) tile(TM{}, t0);
  // 16-row groups left: 0 .. TUM - 1 in every block (rpb is a multiple of 16), up to TUM in
  // the last one (R need not be): a TUM-group remainder runs as a whole tile whose rows past
  // R are clamped on load and dropped on store
  const int tail = (int)((r1 - t0 + 15) / 16);
  if (tail == 1) tile(T1{}, t0);
  if constexpr (TUM > 2) if (tail == 2) tile(T2{}, t0);
  if constexpr (TUM > 3) if (tail == 3) tile(T3{}, t0);
  if constexpr (TUM > 4) if (tail == 4) tile(std::integral_constant<int, 4>{}, t0);
  if constexpr (TUM > 5) if (tail == 5) tile(std::integral_constant<int, 5>{}, t0);
  if constexpr (TUM > 6) if (tail == 6) tile(std::integral_constant<int, 6>{}, t0);
  if constexpr (TUM > 7) if (tail == 7) tile(std::integral_constant<int, 7>{}, t0);
  static_assert(TUM <= 8, "tail tiles");
  if (tail == TUM) tile(TM{}, t0);
}

// split barriers in the one-H-buffer instances but d = 128 (default; there the variant spills
// and measured 4 % slower, d = 192 / 256 / 384 3-4 % faster: profiles/r06/ffn_pp/sb.txt);
// ffn_h3_set_split(0): block barriers everywhere (the labs' A/B switch)
static int g_ffn_split = 1;
void ffn_h3_set_split(int on) { g_ffn_split = on; }

bool ffn_h3_supported(int D, int F) {
  return ((D == 128 || D == 256 || D == 384 || D == 512) && F % 32 == 0 && F >= 32) ||
         (D == 192 && F % 64 == 0 && F >= 64);
}

// the one-accumulator form scales the weight's fp16 hi piece by 2^11: exact below 32
bool ffn_h3_weights_ok(const float* w, long n) {
  for (long i = 0; i < n; ++i)
    if (!(std::fabs(w[i]) < 31.f)) return false;
  return true;
}

// W [rows][cols] f32 -> the two fp16 pieces (hi, lo 2^11), each in ffn_pack_host's order
void ffn_pack_h3_host(const float* w, int rows, int cols, __bf16* out) {
  const size_t n = (size_t)rows * cols;
  std::vector<__bf16> piece(n);
  for (int t = 0; t < 2; ++t) {
    for (size_t i = 0; i < n; ++i) {
      const _Float16 hi = (_Float16)w[i];
      const _Float16 v = t == 0 ? hi : (_Float16)((w[i] - (float)hi) * 2048.f);
      std::memcpy(&piece[i], &v, 2);
    }
    ffn_pack_host(piece.data(), rows, cols, out + t * n);
  }
}

void launch_ffn_fused_h3(float* X, int R, int D, int F, const void* W1, const float* b1,
                         const void* W2, const float* b2, hipStream_t st, const float* byp_orig,
                         const float* byp_scale, const float* Y) {
  if (R <= 0) return;
  if (Y == nullptr) Y = X;
  ZASR_REQUIRE(ffn_h3_supported(D, F), "ffn_fused_h3: unsupported model / feed-forward dim");
  const __bf16* w1 = reinterpret_cast<const __bf16*>(W1);
  const __bf16* w2 = reinterpret_cast<const __bf16*>(W2);
  // one block per CU, rpb rows each (a multiple of 16)
  static int cus[64] = {0};
  int dev = 0;
  ZASR_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    ZASR_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cus[dev] = n > 0 ? n : 256;
  }
  // D = 192: 4 waves (48 output channels each), two blocks per CU
  const int bpc = D == 192 ? 2 : 1;
  const int rpb = 16 * cdiv(cdiv(R, bpc * persist_blocks(cus[dev])), 16);
  const dim3 grid(cdiv(R, rpb));
// SB (split barriers) with one H buffer, EB (batched epilogue loads) but at d = 128: the
// ConvNeXt instance spills with either and measured 4 % / 1.4 % slower (profiles/r06/ffn_pp/)
#define ZASR_FFNH3(DV, TUV, NBV, NWV)                                                                \
  if (NBV == 1 && g_ffn_split && DV != 128)                                                       \
    ZASR_LAUNCH((ffn_wide_h3_kernel<DV, TUV, NBV, NWV, NBV == 1, DV != 128>), grid, dim3(64 * NWV), \
                0, st, X, R, F, w1, b1, w2, b2, byp_orig, byp_scale, rpb, Y);                       \
  else                                                                                             \
    ZASR_LAUNCH((ffn_wide_h3_kernel<DV, TUV, NBV, NWV, false, DV != 128>), grid, dim3(64 * NWV), 0, \
                st, X, R, F, w1, b1, w2, b2, byp_orig, byp_scale, rpb, Y)
  switch (D) {
    // tile rows (16 TUM) / H buffers: the largest tile the LDS and 256 VGPRs hold -- fewer
    // weight passes from L2 and barriers per row, for a barrier per chunk with one H buffer
    // (profiles/r05/ab_s3/ffn_h3_tiles.txt: 4 x 16 rows with two buffers (d = 192: 3 x 16)
    // cost 0.29 ms per hour on the ConvNeXt MLP (d = 128), 0.15 at d = 256, 0.07 at d = 192)
    case 128: ZASR_FFNH3(128, 8, 1, 8); break;
    case 192: ZASR_FFNH3(192, 4, 1, 4); break;
    case 256: ZASR_FFNH3(256, 5, 1, 8); break;
    case 384: ZASR_FFNH3(384, 4, 1, 8); break;
    default: ZASR_FFNH3(512, 3, 2, 8); break;
  }
#undef ZASR_FFNH3
}

// D = 256 in the one-wave-per-32-tokens design compiles to one wave per SIMD (384
// registers) and measured slower than the two GEMMs (tools/ffn_lab.hip); 256..512 use
// ffn_wide_kernel
// W1 [F][D] -> fragments [F/16][D/32][64 lanes][8] and W2 [D][F] -> [D/16][F/32][64][8]:
// element j of lane l of fragment (g, s) is W[16 g + (l & 15)][32 s + 8 (l >> 4) + j]
void ffn_pack_host(const __bf16* w, int rows, int cols, __bf16* out) {
  for (int g = 0; g < rows / 16; ++g)
    for (int s = 0; s < cols / 32; ++s)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j)
          out[(((size_t)g * (cols / 32) + s) * 64 + l) * 8 + j] =
              w[(size_t)(16 * g + (l & 15)) * cols + 32 * s + 8 * (l >> 4) + j];
}

// The rows form (d = 384) is opt-in: ZASR_FFN_ROWS=1 or ffn_set_rows(1).  The kernel alone
// is 1.08-1.10x, but in the pipelined step its 238 resident blocks hold the CUs for a whole
// launch and the search chain on the other stream waits: bench 122.2k vs 123.7k xRT (mean of
// 7 interleaved runs each, profiles/r06/ffn_rows/step_ab.txt).
static int g_ffnw_rows = -1;
void ffn_set_rows(int on) { g_ffnw_rows = on ? 1 : 0; }
int ffn_rows_on() {
  if (g_ffnw_rows < 0) {
    const char* e = getenv("ZASR_FFN_ROWS");
    g_ffnw_rows = e != nullptr && atoi(e) == 1 ? 1 : 0;
  }
  return g_ffnw_rows;
}

bool ffn_fused_supported(int D) {
  return D == 64 || D == 96 || D == 128 || D == 192 || D == 256 || D == 384 || D == 512;
}

void launch_ffn_fused(float* X, int R, int D, int F, const void* W1, const float* b1,
                      const void* W2, const float* b2, hipStream_t st, const float* byp_orig,
                      const float* byp_scale) {
  if (R <= 0) return;
  ZASR_REQUIRE(ffn_fused_supported(D), "ffn_fused: unsupported model dim");
  ZASR_REQUIRE(F % 8 == 0, "ffn_fused: feed-forward dim must be a multiple of 8");
  const __bf16* w1 = reinterpret_cast<const __bf16*>(W1);
  const __bf16* w2 = reinterpret_cast<const __bf16*>(W2);
  if (D >= 256) {
    ZASR_REQUIRE(F % 32 == 0 && F >= 32 && F <= kMaxF,
                 "ffn_fused: feed-forward dim must be a multiple of 32 in [32, 2048] for D >= 256");
    const dim3 grid(cdiv(R, 64));
    static int cus[64] = {0};
    int dev = 0;
    ZASR_HIP_CHECK(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) dev = 0;
    if (cus[dev] == 0) {
      int n = 0;
      ZASR_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
      cus[dev] = n > 0 ? n : 256;
    }
    if (D == 384 && ffn_rows_on()) {
      const int rpb = 16 * cdiv(cdiv(R, persist_blocks(cus[dev])), 16);
      ZASR_LAUNCH((ffn_rows_kernel<384, true>), dim3(cdiv(R, rpb)), dim3(512), 0, st, X, R, F, w1, b1, w2, b2,
                  byp_orig, byp_scale, rpb);
      return;
    }
// EB (batched epilogue loads) at d = 384: 1.5-2 % (profiles/r06/ffn_pp/ffnw_eb.txt); d = 512
// neutral, and at d = 256 it takes the kernel past 128 VGPRs (one block per CU instead of two)
#define ZASR_FFNW(DV) \
  ZASR_LAUNCH((ffn_wide_kernel<DV, DV == 384>), grid, dim3(512), 0, st, X, R, F, w1, b1, w2, b2, byp_orig, byp_scale)
    switch (D) {
      case 256: ZASR_FFNW(256); break;
      case 384: ZASR_FFNW(384); break;
      default: ZASR_FFNW(512); break;
    }
#undef ZASR_FFNW
    return;
  }
  const dim3 grid(cdiv(R, kTok));
#define ZASR_FFN(DV) ZASR_LAUNCH(ffn_fused_kernel<DV>, grid, dim3(256), 0, st, X, R, F, w1, b1, w2, b2, byp_orig, byp_scale)
  switch (D) {
    case 64: ZASR_FFN(64); break;
    case 96: ZASR_FFN(96); break;
    case 128: ZASR_FFN(128); break;
    default: ZASR_FFN(192); break;
  }
#undef ZASR_FFN
}

}  // namespace zasr
