// f16x3 projection GEMM with the activation row tile resident on chip ("h3r"): the f16x3 mode's
// dense projections (attention / conv-module / NonlinAttention in- and out-projections,
// K in {96, 192, 256, 288, 384, 512}) at f32 quality,
//
//   C[m, n] = epi( sum_k A[m, k] W[n, k] + bias[n] )        A f32 [M][K], W [N][K]
//
// The structure is phase A of the fused f16x3 FFN (ffn_kernels.hip ffn_wide_h3_kernel) with an
// epilogue per column chunk instead of phase B: one 8-wave block per CU owns a per-CU share of
// the rows; a 64-128-row tile of A is split once into its two fp16 pieces (hi, lo 2^11) in LDS, and
// the block walks all N columns in chunks of 128 (16 per wave), W's pieces streaming from L2
// in MFMA-fragment order (ffn_pack_h3_host) through a register ring that runs on across chunks
// and tiles.  Products on v_mfma_f32_16x16x32_f16 in the one-accumulator form (w_lo x_hi +
// w_hi x_lo + (w_hi 2^11) x_hi, |w| < 32), so A is read from HBM once and split once (the
// tiled gemm_x3 kernel re-reads and re-splits the A panel for every column tile), no LDS
// traffic for W and no barrier inside a tile: the waves drift freely between their MFMA
// k-loop and their epilogue.  Epilogues NONE, RESADD, GLU.
#include <cmath>

#include "common.h"
#include "gemm.h"

namespace zasr {
namespace {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr float kLo = 2048.f, kLoInv = 1.f / 2048.f;

__device__ __forceinline__ void lds_barrier_h3r() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// the pointers are deliberately not __restrict__: loads from restrict-qualified read-only
// kernel arguments are marked invariant, and the compiler then sinks the ring's prefetches and
// the epilogue's operand loads next to their use (behind a full wait)
struct H3RArgs {
  const float* A;
  const __bf16* W;   // piece 0 (hi); piece 1 at + wpc
  long wpc;
  const float* bias;  // [N] or nullptr
  float* C;
  int ldc;
  int M, N;
  int rpb;                  // rows per block (multiple of 16)
};

#ifdef ZASR_H3R_STAMPS  // development: per-wave stamps of block 0 (tools/h3r_lab.hip)
__device__ long long g_h3r_stamps[8 * 64 * 4];
#define H3R_STAMP(k, i)                                                                        \
  if (blockIdx.x == 0 && lane == 0 && (k) < 64) g_h3r_stamps[(wid * 64 + (k)) * 4 + (i)] = clock64();
#else
#define H3R_STAMP(k, i)
#endif

template <int K, int EPI>
__global__ __launch_bounds__(512, 1) void gemm_h3r_kernel(H3RArgs a) {
  // row stride in halves: 16 (8 j + 2)-byte rows keep the 16x16x32 operand reads conflict-free
  constexpr int XLD = K + (K % 64 == 0 ? 16 : 48);
  // 16-row groups per tile: as many as the LDS (64 XLD bytes per group) and 256 VGPRs hold --
  // each W pass from L2 feeds more rows (profiles/r05/ab_s3/h3r_tiles.txt: enc_gemm -2.4 %
  // vs 4 groups at every K, then -0.7 % from 6 at K = 288 / 384 without RESADD, whose side
  // operands spill there)
  constexpr int TUL = 160 * 1024 / (64 * XLD);
  constexpr int TUMX = K <= 192 ? 8 : (K <= 256 || (K <= 384 && EPI != EPI_RESADD)) ? 6 : 4;
  constexpr int NW = 8, TUM = TUL < TUMX ? TUL : TUMX, TTM = 16 * TUM, CW = 16 * NW;
  static_assert(TUM >= 1 && TUM <= 8, "tile height");
  constexpr int KS = K / 32;
  // W ring depth, a divisor of KS (twice the k-steps in flight measured no better:
  // profiles/r05/gemm_h3r/)
  constexpr int P1 = KS % 3 == 0 ? 3 : 2;
  static_assert(K % 32 == 0, "K must be a multiple of 32");
  __shared__ __attribute__((aligned(16))) _Float16 sX[2][TTM * XLD];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int M = a.M, N = a.N;
  const long r0 = (long)blockIdx.x * a.rpb;
  const long r1 = r0 + a.rpb < M ? r0 + a.rpb : M;
  const int nch = (N + CW - 1) / CW;
  const f16x8 kS = {(_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f,
                    (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f, (_Float16)2048.f};

  // ---- W ring: one stream over (chunk, k-step); groups past N clamp (their output is dropped)
  f16x8 wr[P1][2];
  auto load_w = [&](int c, int s, int slot) {
    const int g = min((c * CW) / 16 + wid, N / 16 - 1);
    const __bf16* p = a.W + ((long)g * KS + s) * 512 + lane * 8;
    wr[slot][0] = *reinterpret_cast<const f16x8*>(p);
    wr[slot][1] = *reinterpret_cast<const f16x8*>(p + a.wpc);
  };
#pragma unroll
  for (int s = 0; s < P1; ++s) load_w(0, s, s);

#ifdef ZASR_H3R_STAMPS
  int kt = 0;  // tiles done (stamps)
#endif
  auto tile = [&](auto tu_c, const long t0, bool first) {
    constexpr int TU = decltype(tu_c)::value, TT = 16 * TU;
    H3R_STAMP(kt, 0)
    if (!first) lds_barrier_h3r();  // every wave is done reading the previous tile
    H3R_STAMP(kt, 1)
    // ---- A tile -> two fp16 piece images (rows past M: a clamped duplicate, never written)
    {
      constexpr int NQ = TT * K / 4, NE = (NQ + 64 * NW - 1) / (64 * NW);  // float4 per thread
      float4 v[NE];
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = min(tid + 64 * NW * i, NQ - 1), row = e / (K / 4), c4 = e - row * (K / 4);
        const long r = t0 + row < M ? t0 + row : M - 1;
        v[i] = *reinterpret_cast<const float4*>(a.A + r * K + 4 * c4);
      }
#pragma unroll
      for (int i = 0; i < NE; ++i) {
        const int e = tid + 64 * NW * i, row = e / (K / 4), c4 = e - row * (K / 4);
        if (NQ % (64 * NW) != 0 && e >= NQ) break;
        const float x4[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        f16x4 hh, ll;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          hh[q] = (_Float16)x4[q];
          ll[q] = (_Float16)((x4[q] - (float)hh[q]) * kLo);
        }
        *reinterpret_cast<f16x4*>(&sX[0][row * XLD + 4 * c4]) = hh;
        *reinterpret_cast<f16x4*>(&sX[1][row * XLD + 4 * c4]) = ll;
      }
    }
    lds_barrier_h3r();
    H3R_STAMP(kt, 2)

    f16x8 xf[2][TU][2];
    auto read_x = [&](int s, int buf) {
#pragma unroll
      for (int u = 0; u < TU; ++u) {
        const int xo = (16 * u + r16) * XLD + 32 * s + 8 * g4;
        xf[buf][u][0] = *reinterpret_cast<const f16x8*>(&sX[0][xo]);
        xf[buf][u][1] = *reinterpret_cast<const f16x8*>(&sX[1][xo]);
      }
    };
    for (int c = 0; c < nch; ++c) {
      const int n0 = c * CW + wid * 16;  // this wave's 16 columns
      const int nc = min(n0, N - 16) + 4 * g4;  // this lane's 4 (clamped for dropped waves)
      // epilogue operands, issued ahead of the k-loop
      f32x4v bv = f32x4v{0.f, 0.f, 0.f, 0.f};
      if (a.bias != nullptr) bv = *reinterpret_cast<const f32x4v*>(a.bias + nc);
      f32x4v side[TU];
      if constexpr (EPI == EPI_RESADD) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const long row = t0 + 16 * u + r16 < M ? t0 + 16 * u + r16 : M - 1;
          side[u] = *reinterpret_cast<const f32x4v*>(a.C + row * a.ldc + nc);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4v acc[TU];
#pragma unroll
      for (int u = 0; u < TU; ++u) acc[u] = f32x4v{0.f, 0.f, 0.f, 0.f};
      read_x(0, 0);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const int slot = s % P1;
        if (s + 1 < KS) read_x(s + 1, (s + 1) & 1);
        const f16x8 wh = wr[slot][0], wl = wr[slot][1];
        const f16x8 ws = wh * kS;
        const int b = s & 1;
#pragma unroll
        for (int u = 0; u < TU; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl, xf[b][u][0], acc[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < TU; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh, xf[b][u][1], acc[u], 0, 0, 0);
#pragma unroll
        for (int u = 0; u < TU; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ws, xf[b][u][0], acc[u], 0, 0, 0);
        // the ring runs on: the last P1 steps issue the next chunk's first ones (after the
        // last chunk: chunk 0, the next tile's)
        if (s + P1 < KS) load_w(c, s + P1, slot);
        else load_w(c + 1 < nch ? c + 1 : 0, s + P1 - KS, slot);
        __builtin_amdgcn_sched_barrier(0);
      }
      // ---- epilogue: lane's row t0 + 16 u + r16, columns n0 + 4 g4 + (0..3) ----
      if (n0 < N) {
#pragma unroll
        for (int u = 0; u < TU; ++u) {
          const long row = t0 + 16 * u + r16;
          if (row >= r1) continue;
          float4 v;
          v.x = acc[u][0] * kLoInv + bv[0];
          v.y = acc[u][1] * kLoInv + bv[1];
          v.z = acc[u][2] * kLoInv + bv[2];
          v.w = acc[u][3] * kLoInv + bv[3];
          if constexpr (EPI == EPI_GLU) {  // interleaved rows (2c, 2c + 1) -> channel c
            *reinterpret_cast<float2*>(a.C + row * a.ldc + nc / 2) =
                make_float2(v.x * sigmoid_fast(v.y), v.z * sigmoid_fast(v.w));
          } else {
            if constexpr (EPI == EPI_RESADD) {
              v.x += side[u][0]; v.y += side[u][1]; v.z += side[u][2]; v.w += side[u][3];
            }
            *reinterpret_cast<float4*>(a.C + row * a.ldc + nc) = v;
          }
        }
      }
    }
    H3R_STAMP(kt, 3)
#ifdef ZASR_H3R_STAMPS
    ++kt;
#endif
  };

  using TM = std::integral_constant<int, TUM>;
  long t0 = r0;
  bool first = true;
  for (; t0 + TTM <= r1; t0 += TTM, first = false) tile(TM{}, t0, first);
  // 16-row groups left: 0 .. TUM - 1 in every block (rpb is a multiple of 16), up to TUM in
  // the last one (M need not be): a TUM-group remainder runs as a whole tile whose rows past
  // M are clamped on load and dropped on store
  const int tail = (int)((r1 - t0 + 15) / 16);
  if (tail == 1) tile(std::integral_constant<int, 1>{}, t0, first);
  if constexpr (TUM > 2) if (tail == 2) tile(std::integral_constant<int, 2>{}, t0, first);
  if constexpr (TUM > 3) if (tail == 3) tile(std::integral_constant<int, 3>{}, t0, first);
  if constexpr (TUM > 4) if (tail == 4) tile(std::integral_constant<int, 4>{}, t0, first);
  if constexpr (TUM > 5) if (tail == 5) tile(std::integral_constant<int, 5>{}, t0, first);
  if constexpr (TUM > 6) if (tail == 6) tile(std::integral_constant<int, 6>{}, t0, first);
  if constexpr (TUM > 7) if (tail == 7) tile(std::integral_constant<int, 7>{}, t0, first);
  if (tail == TUM) tile(TM{}, t0, first);
}

}  // namespace

// K <= 192 with RESADD / GLU stays on gemm_x3: a chunk's k-loop (<= 72 MFMAs per wave) is
// too short to hide the epilogue's C read / store round trip (measured 1.10-1.36x slower on
// the 192-wide stack, profiles/r05/gemm_h3r/)
bool gemm_h3r_supported(int K, int N, int epi) {
  const bool k_ok = K == 96 || K == 192 || K == 256 || K == 288 || K == 384 || K == 512;
  const bool e_ok = epi == EPI_NONE || ((epi == EPI_RESADD || epi == EPI_GLU) && K >= 256);
  return k_ok && e_ok && N >= 128 && N % 16 == 0;
}

void gemm_h3r(const float* A, const void* Wp, const float* bias, float* C, int ldc, int M, int N,
              int K, int epi, hipStream_t st) {
  if (M <= 0) return;
  ZASR_REQUIRE(gemm_h3r_supported(K, N, epi), "gemm_h3r: unsupported shape / epilogue");
  ZASR_REQUIRE(epi != EPI_GLU || ldc * 2 >= N, "gemm_h3r: EPI_GLU writes N / 2 columns");
  ZASR_REQUIRE(ldc % 4 == 0 || (epi == EPI_GLU && ldc % 2 == 0), "gemm_h3r: ldc alignment");
  static int cus[64] = {0};
  int dev = 0;
  ZASR_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    ZASR_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cus[dev] = n > 0 ? n : 256;
  }
  H3RArgs a{A, reinterpret_cast<const __bf16*>(Wp), (long)N * K, bias, C, ldc, M, N,
            16 * cdiv(cdiv(M, persist_blocks(cus[dev])), 16)};
  const dim3 grid(cdiv(M, a.rpb));
#define ZASR_H3R(KV)                                                                      \
  switch (epi) {                                                                          \
    case EPI_RESADD: ZASR_LAUNCH((gemm_h3r_kernel<KV, EPI_RESADD>), grid, dim3(512), 0, st, a); break; \
    case EPI_GLU: ZASR_LAUNCH((gemm_h3r_kernel<KV, EPI_GLU>), grid, dim3(512), 0, st, a); break; \
    default: ZASR_LAUNCH((gemm_h3r_kernel<KV, EPI_NONE>), grid, dim3(512), 0, st, a); break; \
  }
  switch (K) {
    case 96: ZASR_H3R(96); break;
    case 192: ZASR_H3R(192); break;
    case 256: ZASR_H3R(256); break;
    case 288: ZASR_H3R(288); break;
    case 384: ZASR_H3R(384); break;
    default: ZASR_H3R(512); break;
  }
#undef ZASR_H3R
}

}  // namespace zasr
