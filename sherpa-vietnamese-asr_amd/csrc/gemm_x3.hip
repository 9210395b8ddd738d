// Split-bf16 MFMA GEMM ("bf16x3" / "bf16x6" precision modes): near-f32 or f32-quality
// products at bf16 MFMA rates.
//
//   C[m, n] = epi( sum_k A[m, k] * W[n, k] + bias[n] )
//
// Each f32 operand x is carried as NP bf16 pieces, p0 = bf16(x), p1 = bf16(x - p0), ...
// NP = 2: the product is a1 w0 + a0 w1 + a0 w0 in f32 on v_mfma_f32_32x32x16_bf16 (three
// MFMAs where the bf16 mode issues one); the dropped a1 w1 and the two split residuals leave
// ~2^-16 relative per product (bf16 alone: 2^-8): encoder_out ~3e-5 from the fp32 oracle.
// NP = 3: six MFMAs (every a_i w_j with i + j <= 2); what is dropped is below 2^-24, so the
// result is of exact-f32 quality (encoder_out within 4e-6 of the oracle like the exact-f32
// MFMA mode, token-exact; profiles/r03/precision/).  The weights are split once at load;
// the f32 activations are split while staging into LDS.  v_mfma_f32_32x32x2_f32 (the fp32
// mode) runs at 1/16 of the bf16 rate, so six bf16 MFMAs are 2.7x cheaper per product.
//
// Structure follows gemm_bf16_kernel (gemm.hip): BM x BN block tile on 4 waves, BK = 32
// slabs staged through LDS as row-major [row][BK + 8] bf16 images (hi and lo of A and of W),
// two LDS stages, next slab's global loads in registers under the MFMAs (two register sets
// when K is a multiple of 64), tiles numbered so that blocks sharing an A row panel land on
// one XCD, epilogue through LDS as float4 rows.
#include <type_traits>

#include "common.h"
#include "gemm.h"
#include "gemm_dev.h"

namespace zasr {
namespace {

// x -> NP bf16 pieces p0 + p1 (+ p2), each the RNE bf16 of what the previous ones left
template <int NP>
__device__ __forceinline__ void split8(const float4 x0, const float4 x1, bf16x8 (&pc)[NP]) {
  const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
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

// native exp2 / log forms (common.h; ~1e-7 absolute from the libm forms, below the f32
// rounding of the values they feed): the libm log1pf(expf()) pair made the SwooshL-epilogue
// shapes 2-3x slower than the plain ones (profiles/r03/x3_shape_table.json)
// EPI_RESADD with p.byp_orig: the layer's bypass_mid folded in after the residual add,
// launch_bypass's formula (orig + (x - orig) * scale), the same f32 operations in the same
// order, so the result is bit-identical to the separate pass
__device__ __forceinline__ void x3_bypass(const GemmParams& p, float4& v, int row, int col) {
  if (p.byp_orig == nullptr) return;
  const float4 b0 = *reinterpret_cast<const float4*>(p.byp_orig + (long)row * p.ldc + col);
  const float4 k = *reinterpret_cast<const float4*>(p.byp_scale + col);
  v.x = b0.x + (v.x - b0.x) * k.x;
  v.y = b0.y + (v.y - b0.y) * k.y;
  v.z = b0.z + (v.z - b0.z) * k.z;
  v.w = b0.w + (v.w - b0.w) * k.w;
}

template <int EPI>
__device__ __forceinline__ float x3_act(float v) {
  if constexpr (EPI == EPI_SWOOSHL) return swooshl_fast(v);
  if constexpr (EPI == EPI_SWOOSHR) return swooshr_fast(v);
  return v;
}

// NP = 2 ("bf16x3"): pieces (hi, lo), products p0q0 + p0q1 + p1q0 (3 MFMAs), BK = 32.
// NP = 3 ("bf16x6"): pieces (p0, p1, p2), the six products p_i q_j with i + j <= 2 (6 MFMAs,
// dropped terms below 2^-24 relative: exact-f32 quality), BK = 16 (same MFMAs per slab and
// the same LDS as NP = 2).  Weights: piece t at Bw + t * blo.
// FMT 1 ("f16x3"): NP = 2 fp16 pieces, hi + lo * 2^-11 (gemm_dev.h split_h8), the products
// hi*hi into one accumulator and hi*lo + lo*hi into a second, combined in the epilogue.
template <int BM, int BN, int WAVES_M, int WAVES_N, int ALOAD, int EPI, bool DEEP, int NP,
          int BK = (NP == 2 ? 32 : 16), int FMT = 0>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N,
                             FMT == 1 && WAVES_M * WAVES_N <= 4 ? 2 : 1) void gemm_x3_kernel(GemmParams p,
                                                                       const __bf16* Bw, long blo,
                                                                       int tiles_n, int tiles_m) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M;
  constexpr int WTN = BN / WAVES_N;
  constexpr int FM = WTM / 32;
  constexpr int FN = WTN / 32;
  static_assert(FM >= 1 && FN >= 1, "wave tile must be a multiple of 32x32");
  constexpr int LDH = BK + 8;
  constexpr int GPR = BK / 8;
  constexpr int A_G = BM * GPR;
  constexpr int B_G = BN * GPR;
  constexpr int A_LD = (A_G + NT - 1) / NT;
  constexpr int B_LD = (B_G + NT - 1) / NT;
  // stage: A pieces [NP][BM][LDH], then W pieces [NP][BN][LDH]
  constexpr int STAGE = NP * (BM + BN) * LDH;
  constexpr int LDE = 40;
  constexpr int OPER_BYTES = 2 * STAGE * 2;
  constexpr int EPI_BYTES = (NT / 64) * 32 * LDE * 4;
  constexpr int LDS_BYTES = OPER_BYTES > EPI_BYTES ? OPER_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __bf16* const sbase = reinterpret_cast<__bf16*>(smem);

  const float* A = p.A;
  float* C = p.C;
  const float* aux = p.aux;
  int M = p.M, K = p.K, lda = p.lda;
  long b_off = 0;
  const int tiles = tiles_n * tiles_m;
  const int lin = xcd_tile(blockIdx.x, gridDim.x);
  const int zs = lin / tiles;
  if (p.slices) {
    const GemmSlice s = p.slices[zs];
    A += s.a_off;
    b_off = s.b_off;
    C += s.c_off;
    if (aux) aux += s.aux_off;
    M = s.M;
    K = s.K;
    lda = s.lda;
  }
  const __bf16* B = Bw + b_off;
  const int tile = lin - zs * tiles;
  const int m_tile = tile / tiles_n;
  const int m0 = m_tile * BM;
  if (m0 >= M) return;
  const int n0 = (tile - m_tile * tiles_n) * BN;
  const int N = p.N;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WAVES_N;
  const int wn = wid - wm * WAVES_N;

  // k-invariant per-thread row pointers of the dense fast path (rows past M / N clamped)
  const float* arow[A_LD];
  const __bf16* brow[B_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int idx = tid + NT * i;
    const int row = (idx < A_G ? idx : 0) / GPR, k8 = idx % GPR;
    const int gm = m0 + row < M ? m0 + row : M - 1;
    arow[i] = A + (long)gm * lda + 8 * k8;
  }
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int idx = tid + NT * i;
    const int n = (idx < B_G ? idx : 0) / GPR, k8 = idx % GPR;
    const int gn = n0 + n < N ? n0 + n : N - 1;
    brow[i] = B + (long)gn * p.sbn + 8 * k8;
  }

  struct Regs {
    float4 a0[A_LD], a1[A_LD];
    bf16x8 b[NP][B_LD];
  };
  auto gload = [&](Regs& r, int kt) {
    const int k0 = kt * BK;
    if (ALOAD == ALOAD_DENSE && (DEEP || k0 + BK <= K)) {
#pragma unroll
      for (int i = 0; i < A_LD; ++i) {
        r.a0[i] = *reinterpret_cast<const float4*>(arow[i] + k0);
        r.a1[i] = *reinterpret_cast<const float4*>(arow[i] + k0 + 4);
      }
#pragma unroll
      for (int t = 0; t < NP; ++t)
#pragma unroll
        for (int i = 0; i < B_LD; ++i) r.b[t][i] = *reinterpret_cast<const bf16x8*>(brow[i] + t * blo + k0);
      return;
    }
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / GPR, k8 = idx % GPR;
      const int gm = m0 + (idx < A_G ? row : 0), gk = k0 + 8 * k8;
      r.a0[i] = load_a4<ALOAD>(p, A, M, K, lda, gm, gk);
      r.a1[i] = load_a4<ALOAD>(p, A, M, K, lda, gm, gk + 4);
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      const int n = idx / GPR, k8 = idx % GPR;
      const int gn = n0 + n, gk = k0 + 8 * k8;
      const bool ok = idx < B_G && gn < N && gk < K;
      const int nc = gn < N ? gn : N - 1, kc = gk < K ? gk : K - 8;
#pragma unroll
      for (int t = 0; t < NP; ++t) {
        bf16x8 h = *reinterpret_cast<const bf16x8*>(B + t * blo + (long)nc * p.sbn + kc);
        if (!ok) {
#pragma unroll
          for (int q = 0; q < 8; ++q) h[q] = (__bf16)0.f;
        }
        r.b[t][i] = h;
      }
    }
  };
  auto sstore = [&](const Regs& r, int buf) {
    __bf16* As = sbase + buf * STAGE;
    __bf16* Bs = As + NP * BM * LDH;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < A_G) {
        bf16x8 pc[NP];
        const float v[8] = {r.a0[i].x, r.a0[i].y, r.a0[i].z, r.a0[i].w,
                            r.a1[i].x, r.a1[i].y, r.a1[i].z, r.a1[i].w};
        split_fx<FMT, NP>(v, pc);
        const int o = (idx / GPR) * LDH + 8 * (idx % GPR);
#pragma unroll
        for (int t = 0; t < NP; ++t) *reinterpret_cast<bf16x8*>(&As[t * BM * LDH + o]) = pc[t];
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < B_G) {
        const int o = (idx / GPR) * LDH + 8 * (idx % GPR);
#pragma unroll
        for (int t = 0; t < NP; ++t) *reinterpret_cast<bf16x8*>(&Bs[t * BN * LDH + o]) = r.b[t][i];
      }
    }
  };

  f32x16 acc[FM][FN];
  constexpr int FL = FMT == 1 ? FM : 1;  // the lo-product accumulators (FMT 1 only)
  constexpr int FLN = FMT == 1 ? FN : 1;
  f32x16 accl[FL][FLN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < FL; ++i)
#pragma unroll
    for (int j = 0; j < FLN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) accl[i][j][r] = 0.f;

  auto mma_slab = [&](int cur) {
    const __bf16* As = sbase + cur * STAGE;
    const __bf16* Bs = As + NP * BM * LDH;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[NP][FM], b[NP][FN];
      const int kc = ks * 16 + 8 * (lane >> 5);
#pragma unroll
      for (int t = 0; t < NP; ++t) {
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[t][i] = *reinterpret_cast<const bf16x8*>(
              &As[t * BM * LDH + (wm * WTM + i * 32 + (lane & 31)) * LDH + kc]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[t][j] = *reinterpret_cast<const bf16x8*>(
              &Bs[t * BN * LDH + (wn * WTN + j * 32 + (lane & 31)) * LDH + kc]);
      }
      // smallest terms first: for NP = 3, (2,0) (1,1) (0,2) then (1,0) (0,1) then (0,0)
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (FMT == 1) {
            const bf16x8 x[2] = {a[0][i], a[1][i]};
            const bf16x8 y[2] = {b[0][j], b[1][j]};
            mfma_h3(x, y, acc[i][j], accl[i % FL][j % FLN]);
          } else {
#pragma unroll
            for (int sdeg = NP - 1; sdeg >= 0; --sdeg)
#pragma unroll
              for (int u = sdeg; u >= 0; --u)
                acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[u][i], b[sdeg - u][j],
                                                                    acc[i][j], 0, 0, 0);
          }
        }
    }
  };

  const int nkt = (K + BK - 1) / BK;
  if constexpr (DEEP) {
    // dense A, K a multiple of 2 BK (host-checked): two register sets, LDS-only barriers
    // (__syncthreads would drain the slab in flight with vmcnt(0)), slab indices clamped so
    // every load is unconditional and the in-order vmcnt waits stay exact
    Regs x0, x1;
    auto bar = []() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    gload(x0, 0);
    gload(x1, 1);
    sstore(x0, 0);
    bar();
    for (int kt = 0; kt < nkt; kt += 2) {
      gload(x0, min(kt + 2, nkt - 1));
      mma_slab(0);
      sstore(x1, 1);
      bar();
      gload(x1, min(kt + 3, nkt - 1));
      mma_slab(1);
      sstore(x0, 0);
      bar();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  } else {
    Regs r;
    gload(r, 0);
    sstore(r, 0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nkt) gload(r, kt + 1);
      mma_slab(cur);
      if (kt + 1 < nkt) sstore(r, cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: fragment -> LDS (lane: column lane&31, rows (r&3)+8(r>>2)+4(lane>>5)) ->
  // float4 rows (8 lanes per 32-column row); side inputs loaded unconditionally (clamped)
  float* sE = reinterpret_cast<float*>(smem) + wid * (32 * LDE);
  const int c4 = lane & 7;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] =
            FMT == 1 ? acc[i][j][r] + accl[i % FL][j % FLN][r] * kF16LoInv : acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const int col = n0 + wn * WTN + j * 32 + 4 * c4;
      const int cc = col < N ? col : N - 4;
      float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) bias = *reinterpret_cast<const float4*>(p.bias + cc);
      float4 side[4];
      if constexpr (EPI == EPI_RESADD || EPI == EPI_MULAUX) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = m0 + wm * WTM + i * 32 + (lane >> 3) + 8 * q;
          const int rc = row < M ? row : M - 1;
          side[q] = EPI == EPI_RESADD
                        ? *reinterpret_cast<const float4*>(C + (long)rc * p.ldc + cc)
                        : *reinterpret_cast<const float4*>(aux + (long)rc * p.ldaux + cc);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = (lane >> 3) + 8 * q;
        const int row = m0 + wm * WTM + i * 32 + rl;
        float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
        if (row < M && col < N) {
          v.x = x3_act<EPI>(v.x + bias.x);
          v.y = x3_act<EPI>(v.y + bias.y);
          v.z = x3_act<EPI>(v.z + bias.z);
          v.w = x3_act<EPI>(v.w + bias.w);
          if constexpr (EPI == EPI_RESADD) {
            v.x += side[q].x; v.y += side[q].y; v.z += side[q].z; v.w += side[q].w;
            x3_bypass(p, v, row, col);
          }
          if constexpr (EPI == EPI_MULAUX) {
            v.x *= side[q].x; v.y *= side[q].y; v.z *= side[q].z; v.w *= side[q].w;
          }
          if constexpr (EPI == EPI_GLU) {  // columns (2c, 2c + 1) -> channel c
            *reinterpret_cast<float2*>(C + (long)row * p.ldc + col / 2) =
                make_float2(v.x * sigmoid_fast(v.y), v.z * sigmoid_fast(v.w));
          } else {
            *reinterpret_cast<float4*>(C + (long)row * p.ldc + col) = v;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

template <int BM, int BN, int WM, int WN, int ALOAD, int EPI, int NP, int BK = (NP == 2 ? 32 : 16),
          int FMT = 0>
void launch_x3_t(const GemmParams& p, const __bf16* Bw, long blo, hipStream_t st) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.max_M, BM);
  dim3 grid(tn * tm * (p.slices ? p.num_slices : 1));
  if (ALOAD == ALOAD_DENSE && !p.slices && p.K % (2 * BK) == 0 && p.lda % 4 == 0) {
    ZASR_LAUNCH((gemm_x3_kernel<BM, BN, WM, WN, ALOAD, EPI, true, NP, BK, FMT>), grid,
                       dim3(64 * WM * WN), 0, st, p, Bw, blo, tn, tm);
    return;
  }
  ZASR_LAUNCH((gemm_x3_kernel<BM, BN, WM, WN, ALOAD, EPI, false, NP, BK, FMT>), grid,
                     dim3(64 * WM * WN), 0, st, p, Bw, blo, tn, tm);
}

// ---------------------------------------------------------------------------------------
// f16x3 on the LDS-DMA pipeline (dense A, K % 32 == 0, no z-slices): every operand byte
// reaches LDS by global_load_lds (16 B per lane, no VGPR staging, no ds_write): the f32 A
// slab (128 rows x 32 k, rows swizzled as gemm.hip's gemm_glds_kernel: 16-byte chunk c of row
// r at chunk c ^ ((r >> 1) & 7)) and the two fp16 piece images of W (BN rows x 32 k each,
// chunk c of row r at c ^ ((r >> 2) & 3)); NS stages, NS - 2 slabs in flight across the raw
// barrier.  Each wave splits its A fragments into (hi, lo) at the fragment read (VALU beside
// the MFMAs) and issues hi*hi into one accumulator, hi*lo + lo*hi into the other.
// 4 waves, wave tile 64 x BN/2.
// ---------------------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void* h3_lds_t;

// f16x3 epilogue of the LDS-DMA kernels (gemm_x3_kernel's): per 32 x 32 fragment, hi + lo *
// 2^-11 -> the wave's LDS slice sE (32 x 40 floats) -> float4 rows with bias, activation and
// the side input (rows clamped for the side loads, stores guarded).  row0 / col0: the wave's
// first output row / column.
template <int EPI, int FM, int FN>
__device__ __forceinline__ void h3_epilogue(const GemmParams& p, float* sE,
                                            const f32x16 (&acc)[FM][FN],
                                            const f32x16 (&accl)[FM][FN], int row0, int col0,
                                            int lane) {
  constexpr int LDE = 40;
  const int M = p.M, N = p.N;
  const int r32 = lane & 31, h = lane >> 5, c4 = lane & 7;
  float* C = p.C;
  const float* aux = p.aux;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sE[((r & 3) + 8 * (r >> 2) + 4 * h) * LDE + r32] = acc[i][j][r] + accl[i][j][r] * kF16LoInv;
      __builtin_amdgcn_wave_barrier();
      const int col = col0 + j * 32 + 4 * c4;
      const int cc = col < N ? col : N - 4;
      float4 bias = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias) bias = *reinterpret_cast<const float4*>(p.bias + cc);
      float4 side[4];
      if constexpr (EPI == EPI_RESADD || EPI == EPI_MULAUX) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = row0 + i * 32 + (lane >> 3) + 8 * q;
          const int rc = row < M ? row : M - 1;
          side[q] = EPI == EPI_RESADD
                        ? *reinterpret_cast<const float4*>(C + (long)rc * p.ldc + cc)
                        : *reinterpret_cast<const float4*>(aux + (long)rc * p.ldaux + cc);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = (lane >> 3) + 8 * q;
        const int row = row0 + i * 32 + rl;
        float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
        if (row < M && col < N) {
          v.x = x3_act<EPI>(v.x + bias.x);
          v.y = x3_act<EPI>(v.y + bias.y);
          v.z = x3_act<EPI>(v.z + bias.z);
          v.w = x3_act<EPI>(v.w + bias.w);
          if constexpr (EPI == EPI_RESADD) {
            v.x += side[q].x; v.y += side[q].y; v.z += side[q].z; v.w += side[q].w;
            x3_bypass(p, v, row, col);
          }
          if constexpr (EPI == EPI_MULAUX) {
            v.x *= side[q].x; v.y *= side[q].y; v.z *= side[q].z; v.w *= side[q].w;
          }
          if constexpr (EPI == EPI_GLU) {  // columns (2c, 2c + 1) -> channel c
            *reinterpret_cast<float2*>(C + (long)row * p.ldc + col / 2) =
                make_float2(v.x * sigmoid_fast(v.y), v.z * sigmoid_fast(v.w));
          } else {
            *reinterpret_cast<float4*>(C + (long)row * p.ldc + col) = v;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// PR = 1: the hi x hi product only (a diagnostic of the split_lab: what the loop costs
// without the two correction MFMAs; not numerically a split GEMM)
// ALD = ALOAD_CONV3 (Conv2dSubsampling's conv.7 as an implicit GEMM, K = 9 taps x 32
// channels): k-tile kt is tap kt, so every A row segment is 32 contiguous channels of the
// conv.4 output at a row-independent tap offset -- the same 128-byte LDS-DMA pieces as the
// dense case from gathered row bases (load_a4<ALOAD_CONV3>'s addresses)
template <int NS, int EPI, int BN, int WM = 2, int PR = 3, int ALD = ALOAD_DENSE, int RB = 0>
__global__ __launch_bounds__(256, NS == 2 ? 2 : 1) void gemm_glds_h3_kernel(GemmParams p,
                                                                          const __bf16* Bw,
                                                                          long blo, int tiles_n,
                                                                          int tiles_m) {
  constexpr int BM = 128, BK = 32;
  // WM x WN waves: WM = 4 gives each wave all BN columns of 32 rows, so every A element is
  // split by one wave (WM = 2: by two)
  constexpr int WN = 4 / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 4;
  constexpr int B_BYTES = BN * BK * 2;  // one piece
  constexpr int STAGE = A_BYTES + 2 * B_BYTES;
  constexpr int GA = A_BYTES / 1024 / 4;
  constexpr int GB = B_BYTES / 1024 / 4;
  constexpr int G = GA + 2 * GB;
  constexpr int LDE = 40;
  constexpr int EPI_BYTES = 4 * 32 * LDE * 4;
  constexpr int LDS_BYTES = NS * STAGE > EPI_BYTES ? NS * STAGE : EPI_BYTES;
  static_assert(NS >= 2 && NS <= 3, "stages");
  static_assert(B_BYTES % 4096 == 0, "BN must be a multiple of 64");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS_BYTES];

  // z-slices (per-sequence GEMMs, e.g. conv.7): tiles_n x tiles_m tiles per slice, the
  // slice's operand offsets and M / K / lda applied to a local copy of the parameters
  GemmParams q = p;
  const int lin = xcd_tile(blockIdx.x, gridDim.x);
  const int per = tiles_n * tiles_m;
  const int zs = lin / per;
  const int tile = lin - zs * per;
  if (q.slices) {
    const GemmSlice sl = q.slices[zs];
    q.A += sl.a_off;
    q.C += sl.c_off;
    if (q.aux) q.aux += sl.aux_off;
    q.M = sl.M;
    q.K = sl.K;
    q.lda = sl.lda;
    Bw += sl.b_off;
  }
  const float* A = q.A;
  const int M = q.M, K = q.K, lda = q.lda, N = q.N;
  const int m_tile = tile / tiles_n;
  const int m0 = m_tile * BM;
  if (m0 >= M) return;  // a slice shorter than the longest (whole block)
  const int n0 = (tile - m_tile * tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nkt = K / BK;

  const float* asrc[GA];
  const __bf16* bsrc[GB];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int row = (wid * GA + g) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    const int gr = m0 + row < M ? m0 + row : M - 1;
    if constexpr (ALD == ALOAD_CONV3) {
      const int t = gr / 19, f = gr - t * 19;
      asrc[g] = A + ((long)t * 39 + 2 * f) * 32 + 4 * lc;
    } else {
      asrc[g] = A + (long)gr * lda + 4 * lc;
    }
  }
#pragma unroll
  for (int g = 0; g < GB; ++g) {
    const int row = (wid * GB + g) * 16 + (lane >> 2);
    const int lc = (lane & 3) ^ ((row >> 2) & 3);
    const int gn = n0 + row < N ? n0 + row : N - 1;
    bsrc[g] = Bw + (long)gn * p.sbn + 8 * lc;
  }
  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NS) * STAGE;
    const int k0 = kt * BK;
    // A offset of k-tile kt: dense k0; conv.7 tap kt = (kt / 3, kt % 3) of (time, freq)
    const long ak = ALD == ALOAD_CONV3 ? ((long)(kt / 3) * 39 + kt % 3) * 32 : k0;
#pragma unroll
    for (int g = 0; g < GA; ++g)
      __builtin_amdgcn_global_load_lds(const_cast<float*>(asrc[g] + ak),
                                       (h3_lds_t)(st + (wid * GA + g) * 1024), 16, 0, 0);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < GB; ++g)
        __builtin_amdgcn_global_load_lds(const_cast<__bf16*>(bsrc[g] + t * blo + k0),
                                         (h3_lds_t)(st + A_BYTES + t * B_BYTES + (wid * GB + g) * 1024),
                                         16, 0, 0);
  };

  f32x16 acc[FM][FN], accl[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = accl[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkt) issue(s);
  const int r32 = lane & 31, h = lane >> 5;
  for (int kt = 0; kt < nkt; ++kt) {
    if constexpr (NS == 3) {
      if (kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const unsigned char* st = smem + (kt % NS) * STAGE;
    // fragments of k-step ks (16 deep): A rows split into fp16 hi / lo, B pieces as stored
    auto frags = [&](int ks, bf16x8 (&a)[FM][2], bf16x8 (&b)[FN][2]) {
      const int ch = 2 * ks + h;
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int row = wm * WTM + i * 32 + r32;
        const int sw = (row >> 1) & 7;
        const float4 x0 = *reinterpret_cast<const float4*>(st + row * 128 + (((2 * ch) ^ sw) << 4));
        const float4 x1 = *reinterpret_cast<const float4*>(st + row * 128 + (((2 * ch + 1) ^ sw) << 4));
        const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
        split_h8(v, a[i]);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int row = wn * WTN + j * 32 + r32;
        const int off = row * 64 + ((ch ^ ((row >> 2) & 3)) << 4);
        b[j][0] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + off);
        b[j][1] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + B_BYTES + off);
      }
    };
    auto products = [&](const bf16x8 (&a)[FM][2], const bf16x8 (&b)[FN][2]) {
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr (PR == 1)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                __builtin_bit_cast(f16x8, a[i][0]), __builtin_bit_cast(f16x8, b[j][0]), acc[i][j],
                0, 0, 0);
          else
            mfma_h3(a[i], b[j], acc[i][j], accl[i][j]);
        }
    };
    if constexpr (RB) {
      // every fragment of the stage read before the next stage's DMA goes out: an LDS read
      // behind an LDS-DMA makes the compiler wait for the DMA (vmcnt(0)), which put a full
      // memory round trip in front of every k-tile's MFMAs
      bf16x8 a[2][FM][2], b[2][FN][2];
      frags(0, a[0], b[0]);
      frags(1, a[1], b[1]);
      if (kt + NS - 1 < nkt) issue(kt + NS - 1);
      products(a[0], b[0]);
      products(a[1], b[1]);
    } else {
      if (kt + NS - 1 < nkt) issue(kt + NS - 1);  // the stage every wave finished reading
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[FM][2], b[FN][2];
        frags(ks, a, b);
        products(a, b);
      }
    }
  }
  __syncthreads();

  h3_epilogue<EPI, FM, FN>(q, reinterpret_cast<float*>(smem) + wid * (32 * LDE), acc, accl,
                           m0 + wm * WTM, n0 + wn * WTN, lane);
}

template <int NS, int EPI, int BN, int WM = 2, int PR = 3, int ALD = ALOAD_DENSE, int RB = 0>
void launch_glds_h3(const GemmParams& p, const __bf16* Bw, long blo, hipStream_t st) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.slices ? p.max_M : p.M, 128);
  ZASR_LAUNCH((gemm_glds_h3_kernel<NS, EPI, BN, WM, PR, ALD, RB>),
                     dim3(tn * tm * (p.slices ? p.num_slices : 1)), dim3(256), 0, st, p, Bw, blo,
                     tn, tm);
}

// fp16 pieces (FMT 1).  The LDS-DMA kernel wherever its operand layout fits; the register-
// staged kernel (BK = 16: two stages at 41 KB of LDS, 3 blocks per CU) for the rest.  (The
// round-4 2 x 2-wave LDS-DMA layouts, the register-A and deep-ring variants measured slower and
// are gone; NonlinAttention runs fused in the attention kernel in this mode, so
// no z-sliced dense GEMM reaches here.)
template <int ALOAD, int EPI>
void launch_h3(const GemmParams& p, const __bf16* Bw, long blo, hipStream_t st) {
  if constexpr (ALOAD == ALOAD_CONV3) {
    // (z-sliced launches carry K in the slices; the conv.7 loader's K is 9 taps x 32 = 288)
    if ((p.slices ? p.max_M > 0 : p.K == 288 && p.M >= 128) && p.N % 128 == 0 && p.sbn == 288)
      return launch_glds_h3<2, EPI, 128, 4, 3, ALOAD_CONV3, 1>(p, Bw, blo, st);
  }
  if constexpr (ALOAD == ALOAD_DENSE) {
    // any N % 4 == 0: the B rows past N are clamped loads, the epilogue stores col < N only
    // (the attention in-projections: N = 68 H = 272 / 544, the value projection 12 H = 48)
    if (!p.slices && p.K % 32 == 0 && p.lda % 4 == 0 && p.sbn % 8 == 0 && p.M >= 128 &&
        p.N % 4 == 0) {
      // 4 x 1 waves (each A element split by one wave), the stage's fragments read before
      // the next stage's DMA (split_lab_tiles_v7: 0.28-0.34 of the fp16 peak on the FFN /
      // projection shapes vs 0.24-0.27 for the 2 x 2 loop that issued first)
      const bool w128 = cdiv(p.N, 128) * 128 * 10 <= cdiv(p.N, 64) * 64 * 11;
      if (w128) return launch_glds_h3<2, EPI, 128, 4, 3, ALOAD_DENSE, 1>(p, Bw, blo, st);
      return launch_glds_h3<2, EPI, 64, 4, 3, ALOAD_DENSE, 1>(p, Bw, blo, st);
    }
  }
  const int pad128 = cdiv(p.N, 128) * 128, pad64 = cdiv(p.N, 64) * 64, pad32 = cdiv(p.N, 32) * 32;
  const int BN = (pad128 * 100 <= pad32 * 115) ? 128 : (pad64 * 100 <= pad32 * 115 ? 64 : 32);
  const long blocks128 = (long)cdiv(p.max_M, 128) * cdiv(p.N, BN) * (p.slices ? p.num_slices : 1);
  const bool big = blocks128 >= 512;
  if (BN == 128) {
    if (big) launch_x3_t<128, 128, 2, 2, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
    else launch_x3_t<64, 128, 2, 2, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
  } else if (BN == 64) {
    if (big) launch_x3_t<128, 64, 2, 2, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
    else launch_x3_t<64, 64, 2, 2, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
  } else {
    if (big) launch_x3_t<128, 32, 4, 1, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
    else launch_x3_t<64, 32, 2, 1, ALOAD, EPI, 2, 16, 1>(p, Bw, blo, st);
  }
}

template <int ALOAD, int EPI, int NP>
void launch_x3(const GemmParams& p, const __bf16* Bw, long blo, hipStream_t st) {
  // BN: the largest of {128, 64, 32} whose padded width is within 15 % of the tightest
  const int pad128 = cdiv(p.N, 128) * 128, pad64 = cdiv(p.N, 64) * 64, pad32 = cdiv(p.N, 32) * 32;
  const int BN = (pad128 * 100 <= pad32 * 115) ? 128 : (pad64 * 100 <= pad32 * 115 ? 64 : 32);
  const long blocks128 = (long)cdiv(p.max_M, 128) * cdiv(p.N, BN) * (p.slices ? p.num_slices : 1);
  const bool big = blocks128 >= 512;
  // 8-wave 128 x 256 / 256 x 128 tiles were 10-20 % faster alone (tools/x6_bench,
  // profiles/r03/split_gemm/x6_tile_lab_v1.txt) but slower under the batch pipeline, where
  // two encoder streams share the CUs (enc_gemm 55.7 -> 58.4 ms per step): 4-wave tiles
  if (BN == 128) {
    if (big) launch_x3_t<128, 128, 2, 2, ALOAD, EPI, NP>(p, Bw, blo, st);
    else launch_x3_t<64, 128, 2, 2, ALOAD, EPI, NP>(p, Bw, blo, st);
  } else if (BN == 64) {
    if (big) launch_x3_t<128, 64, 2, 2, ALOAD, EPI, NP>(p, Bw, blo, st);
    else launch_x3_t<64, 64, 2, 2, ALOAD, EPI, NP>(p, Bw, blo, st);
  } else {
    if (big) launch_x3_t<128, 32, 4, 1, ALOAD, EPI, NP>(p, Bw, blo, st);
    else launch_x3_t<64, 32, 2, 1, ALOAD, EPI, NP>(p, Bw, blo, st);
  }
}

// NP = 2 / 3: bf16 pieces; NP = kPiecesF16 (4): the two fp16 pieces of the f16x3 format
template <int NP>
void gemm_split_dispatch(const GemmParams& p, const __bf16* B, long b_lo, int epi, int aload,
                         hipStream_t st) {
#define ZASR_X3(AL, EP)                                  \
  do {                                                   \
    if constexpr (NP == kPiecesF16)                      \
      return launch_h3<AL, EP>(p, B, b_lo, st);          \
    else                                                 \
      return launch_x3<AL, EP, NP>(p, B, b_lo, st);      \
  } while (0)
  if (aload == ALOAD_DENSE) {
    switch (epi) {
      case EPI_NONE: ZASR_X3(ALOAD_DENSE, EPI_NONE);
      case EPI_SWOOSHL: ZASR_X3(ALOAD_DENSE, EPI_SWOOSHL);
      case EPI_SWOOSHR: ZASR_X3(ALOAD_DENSE, EPI_SWOOSHR);
      case EPI_RESADD: ZASR_X3(ALOAD_DENSE, EPI_RESADD);
      case EPI_MULAUX: ZASR_X3(ALOAD_DENSE, EPI_MULAUX);
      case EPI_GLU: ZASR_X3(ALOAD_DENSE, EPI_GLU);
      default: break;
    }
  } else if (aload == ALOAD_CONV2 && epi == EPI_SWOOSHR) {
    ZASR_X3(ALOAD_CONV2, EPI_SWOOSHR);
  } else if (aload == ALOAD_CONV3 && epi == EPI_SWOOSHR) {
    ZASR_X3(ALOAD_CONV3, EPI_SWOOSHR);
  }
#undef ZASR_X3
  throw std::runtime_error("gemm_x3: unsupported (aload, epi) combination");
}

__global__ void split_bf16_kernel(const float* __restrict__ src, __bf16* __restrict__ dst,
                                  long n, int pieces) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    float r = src[i];
    if (pieces == kPiecesF16) {  // fp16 hi, fp16 (x - hi) * 2^11 (gemm_dev.h split_h8)
      const _Float16 h = (_Float16)r;
      const _Float16 l = (_Float16)((r - (float)h) * kF16Lo);
      reinterpret_cast<_Float16*>(dst)[i] = h;
      reinterpret_cast<_Float16*>(dst)[n + i] = l;
      return;
    }
    for (int t = 0; t < pieces; ++t) {
      const __bf16 h = (__bf16)r;
      dst[t * n + i] = h;
      r -= (float)h;
    }
  }
}

}  // namespace

void gemm_x3(const GemmParams& p, const void* Bw, long b_lo, int epi, int aload, hipStream_t st,
             int pieces) {
  ZASR_REQUIRE(p.N > 0, "gemm_x3: N must be positive");
  if (p.max_M <= 0) return;
  ZASR_REQUIRE(p.N % 4 == 0 && p.ldc % 4 == 0 && (epi != EPI_MULAUX || p.ldaux % 4 == 0),
               "gemm_x3: N and the C / aux row strides must be multiples of 4");
  ZASR_REQUIRE(epi != EPI_GLU || (p.ldc * 2 >= p.N && p.ldc % 2 == 0),
               "gemm_x3: EPI_GLU writes N / 2 columns");
  ZASR_REQUIRE(p.slices != nullptr || (p.K % 8 == 0 && p.lda % 4 == 0),
               "gemm_x3: K must be a multiple of 8 and lda of 4");
  ZASR_REQUIRE(pieces == 2 || pieces == 3 || pieces == kPiecesF16,
               "gemm_x3: pieces must be 2, 3 or kPiecesF16");
  const __bf16* B = reinterpret_cast<const __bf16*>(Bw);
  if (pieces == 2)
    gemm_split_dispatch<2>(p, B, b_lo, epi, aload, st);
  else if (pieces == 3)
    gemm_split_dispatch<3>(p, B, b_lo, epi, aload, st);
  else
    gemm_split_dispatch<kPiecesF16>(p, B, b_lo, epi, aload, st);
}

void split_to_bf16(const float* src, void* dst, long n, int pieces, hipStream_t st) {
  if (n <= 0) return;
  ZASR_LAUNCH(split_bf16_kernel, dim3(cdivl(n, 256)), dim3(256), 0, st, src,
                     reinterpret_cast<__bf16*>(dst), n, pieces);
}

}  // namespace zasr
