// GEMM ablation lab (development tool, not part of libzasr).  Times the production bf16 GEMM
// (csrc/gemm.hip, launch_tile_h) on the Zipformer-68M stack-0 shapes, and an ablated copy of
// its main loop with parts switched off (DBG bits: 1 = no epilogue stores, 2 = no MFMA,
// 4 = no A global loads) to see which resource bounds each shape.
// Build: make -C tools gemm_lab ; run on the GPU box: tools/gemm_lab
#include "../csrc/gemm.hip"

#include <cstdio>
#include <vector>

using namespace zasr;

namespace lab {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int BM, int BN, int BK, int WAVES_M, int WAVES_N, typename TA, typename TC, int DBG>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N) void k(GemmParams p, const __bf16* Bw,
                                                           int tiles_n) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N, FM = WTM / 32, FN = WTN / 32;
  constexpr int LDH = BK + 8, GPR = BK / 8, A_G = BM * GPR, B_G = BN * GPR;
  constexpr int A_LD = (A_G + NT - 1) / NT, B_LD = (B_G + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LDH;
  constexpr int LDE = 40;
  constexpr int OPER_BYTES = 2 * STAGE * 2, EPI_BYTES = (NT / 64) * 32 * LDE * 4;
  constexpr int LDS_BYTES = OPER_BYTES > EPI_BYTES ? OPER_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __bf16* const sbase = reinterpret_cast<__bf16*>(smem);
  const TA* A = reinterpret_cast<const TA*>(p.A);
  TC* C = reinterpret_cast<TC*>(p.C);
  const int M = p.M, K = p.K, lda = p.lda, N = p.N;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int m_tile = tile / tiles_n;
  const int m0 = m_tile * BM;
  if (m0 >= M) return;
  const int n0 = (tile - m_tile * tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid - wm * WAVES_N;
  bf16x8 ra[A_LD], rb[B_LD];
  constexpr bool FULLA = (DBG & 8) != 0 && sizeof(TA) == 4;
  constexpr int PPR = BK / 4;                 // 16-byte f32 pieces per row slab
  constexpr int A_P = BM * PPR;
  constexpr int A_LP = (A_P + NT - 1) / NT;
  float4 rf[FULLA ? A_LP : 1];
  auto gload = [&](int kt) {
    if constexpr (FULLA) {
#pragma unroll
      for (int i = 0; i < A_LP; ++i) {
        const int idx = tid + NT * i;
        const int row = idx / PPR, k4 = idx % PPR;
        int gm = m0 + row, gk = kt * BK + 4 * k4;
        const bool ok = gm < M && gk < K;
        gm = gm < M ? gm : M - 1;
        gk = gk < K ? gk : K - 4;
        const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(A) + (long)gm * lda + gk);
        rf[i] = ok ? v : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < (FULLA ? 0 : A_LD); ++i) {
      const int idx = tid + NT * i;
      const int row = idx / GPR, k8 = idx % GPR;
      if constexpr ((DBG & 4) != 0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) ra[i][q] = (__bf16)(float)(row + kt);
      } else {
        ra[i] = load_a8<ALOAD_DENSE, TA>(p, A, M, K, lda, m0 + (idx < A_G ? row : 0), kt * BK + 8 * k8);
      }
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      const int n = idx / GPR, k8 = idx % GPR;
      const int gn = n0 + n, gk = kt * BK + 8 * k8;
      const int nc = gn < N ? gn : N - 1, kc = gk < K ? gk : K - 8;
      rb[i] = *reinterpret_cast<const bf16x8*>(Bw + (long)nc * p.sbn + kc);
    }
  };
  auto sstore = [&](int buf) {
    __bf16* As = sbase + buf * STAGE;
    __bf16* Bs = As + BM * LDH;
    if constexpr (FULLA) {
#pragma unroll
      for (int i = 0; i < A_LP; ++i) {
        const int idx = tid + NT * i;
        if (idx < A_P) {
          bf16x4 h;
          h[0] = (__bf16)rf[i].x; h[1] = (__bf16)rf[i].y; h[2] = (__bf16)rf[i].z; h[3] = (__bf16)rf[i].w;
          *reinterpret_cast<bf16x4*>(&As[(idx / PPR) * LDH + 4 * (idx % PPR)]) = h;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < (FULLA ? 0 : A_LD); ++i) {
      const int idx = tid + NT * i;
      if (idx < A_G) *reinterpret_cast<bf16x8*>(&As[(idx / GPR) * LDH + 8 * (idx % GPR)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < B_G) *reinterpret_cast<bf16x8*>(&Bs[(idx / GPR) * LDH + 8 * (idx % GPR)]) = rb[i];
    }
  };
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nkt = (K + BK - 1) / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) gload(kt + 1);
    const __bf16* As = sbase + cur * STAGE;
    const __bf16* Bs = As + BM * LDH;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          if constexpr ((DBG & 2) != 0)
            acc[i][j][0] += (float)a[i][0] * (float)b[j][0];
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
    }
    if (kt + 1 < nkt) sstore(cur ^ 1);
    __syncthreads();
  }
  float* sE = reinterpret_cast<float*>(smem) + wid * (32 * LDE);
  const int c4 = lane & 7;
  if constexpr ((DBG & 16) != 0 && !std::is_same<TC, float>::value) {
    // 16-byte bf16 stores: lane -> row (lane >> 2) + 16 q, columns 8 (lane & 3) .. + 7
    const int c8 = lane & 3;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] = acc[i][j][r];
        __builtin_amdgcn_wave_barrier();
        const int col = n0 + wn * WTN + j * 32 + 8 * c8;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int rl = (lane >> 2) + 16 * q;
          const int row = m0 + wm * WTM + i * 32 + rl;
          const float4 v0 = *reinterpret_cast<const float4*>(&sE[rl * LDE + 8 * c8]);
          const float4 v1 = *reinterpret_cast<const float4*>(&sE[rl * LDE + 8 * c8 + 4]);
          if (row < M && col < N) {
            bf16x8 h;
            h[0] = (__bf16)v0.x; h[1] = (__bf16)v0.y; h[2] = (__bf16)v0.z; h[3] = (__bf16)v0.w;
            h[4] = (__bf16)v1.x; h[5] = (__bf16)v1.y; h[6] = (__bf16)v1.z; h[7] = (__bf16)v1.w;
            *reinterpret_cast<bf16x8*>(C + (long)row * p.ldc + col) = h;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const int col = n0 + wn * WTN + j * 32 + 4 * c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = (lane >> 3) + 8 * q;
        const int row = m0 + wm * WTM + i * 32 + rl;
        float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
        if (row < M && col < N) {
          TC* dst = C + (long)row * p.ldc + col;
          if constexpr ((DBG & 1) != 0) {
            if (v.x == 12345.678f) *reinterpret_cast<float*>(C) = v.y;
          } else if constexpr (std::is_same<TC, float>::value) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            bf16x4 h;
            h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
            *reinterpret_cast<bf16x4*>(dst) = h;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
}

// persistent variant: grid G (multiple of 8); XCD group x = b % 8 owns a contiguous tile range,
// its blocks stride through it; the next tile's first K-slab is loaded under the epilogue
template <int BM, int BN, int BK, int WAVES_M, int WAVES_N, typename TA, typename TC>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N) void kp(GemmParams p, const __bf16* Bw,
                                                            int tiles_n, int ntiles) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N, FM = WTM / 32, FN = WTN / 32;
  constexpr int LDH = BK + 8, GPR = BK / 8, A_G = BM * GPR, B_G = BN * GPR;
  constexpr int A_LD = (A_G + NT - 1) / NT, B_LD = (B_G + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LDH;
  constexpr int LDE = 40;
  constexpr int OPER_BYTES = 2 * STAGE * 2, EPI_BYTES = (NT / 64) * 32 * LDE * 4;
  // epilogue scratch does not alias the stage buffers (the next tile's slab 0 lands there)
  __shared__ __attribute__((aligned(16))) unsigned char smem[OPER_BYTES + EPI_BYTES];
  __bf16* const sbase = reinterpret_cast<__bf16*>(smem);
  const TA* A = reinterpret_cast<const TA*>(p.A);
  TC* C = reinterpret_cast<TC*>(p.C);
  const int M = p.M, K = p.K, lda = p.lda, N = p.N;
  const int G = gridDim.x, xg = blockIdx.x & 7, slot = blockIdx.x >> 3, per_g = G >> 3;
  const int per = ntiles >> 3, rem = ntiles & 7;
  const int t_begin = xg < rem ? xg * (per + 1) : rem * (per + 1) + (xg - rem) * per;
  const int t_end = t_begin + per + (xg < rem ? 1 : 0);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid - wm * WAVES_N;
  bf16x8 ra[A_LD], rb[B_LD];
  auto gload = [&](int m0, int n0, int kt) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / GPR, k8 = idx % GPR;
      ra[i] = load_a8<ALOAD_DENSE, TA>(p, A, M, K, lda, m0 + (idx < A_G ? row : 0), kt * BK + 8 * k8);
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      const int n = idx / GPR, k8 = idx % GPR;
      const int gn = n0 + n, gk = kt * BK + 8 * k8;
      const int nc = gn < N ? gn : N - 1, kc = gk < K ? gk : K - 8;
      rb[i] = *reinterpret_cast<const bf16x8*>(Bw + (long)nc * p.sbn + kc);
    }
  };
  auto sstore = [&](int buf) {
    __bf16* As = sbase + buf * STAGE;
    __bf16* Bs = As + BM * LDH;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < A_G) *reinterpret_cast<bf16x8*>(&As[(idx / GPR) * LDH + 8 * (idx % GPR)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < B_G) *reinterpret_cast<bf16x8*>(&Bs[(idx / GPR) * LDH + 8 * (idx % GPR)]) = rb[i];
    }
  };
  const int nkt = (K + BK - 1) / BK;
  int t = t_begin + slot;
  if (t >= t_end) return;
  gload((t / tiles_n) * BM, (t % tiles_n) * BN, 0);
  for (; t < t_end; t += per_g) {
    const int m_tile = t / tiles_n;
    const int m0 = m_tile * BM, n0 = (t - m_tile * tiles_n) * BN;
    sstore(0);
    __syncthreads();
    f32x16 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nkt) gload(m0, n0, kt + 1);
      else if (t + per_g < t_end) {
        const int tn = t + per_g;
        gload((tn / tiles_n) * BM, (tn % tiles_n) * BN, 0);  // next tile, under the epilogue
      }
      const __bf16* As = sbase + cur * STAGE;
      const __bf16* Bs = As + BM * LDH;
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nkt) sstore(cur ^ 1);
      __syncthreads();
    }
    float* sE = reinterpret_cast<float*>(smem + OPER_BYTES) + wid * (32 * LDE);
    const int c4 = lane & 7;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] = acc[i][j][r];
        __builtin_amdgcn_wave_barrier();
        const int col = n0 + wn * WTN + j * 32 + 4 * c4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = (lane >> 3) + 8 * q;
          const int row = m0 + wm * WTM + i * 32 + rl;
          float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
          if (row < M && col < N) {
            TC* dst = C + (long)row * p.ldc + col;
            if constexpr (std::is_same<TC, float>::value) {
              *reinterpret_cast<float4*>(dst) = v;
            } else {
              bf16x4 h;
              h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
              *reinterpret_cast<bf16x4*>(dst) = h;
            }
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
  }
}

// whole-K variant (K <= KMAX): the block's A rows [BM x K] are one contiguous chunk, streamed
// with consecutive 16-byte pieces per lane (full cache lines), converted to bf16 into LDS;
// B [BN x K] likewise; then all MFMAs; epilogue as above.
template <int BM, int BN, int KMAX, int WAVES_M, int WAVES_N, typename TA, typename TC>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N) void kf(GemmParams p, const __bf16* Bw,
                                                            int tiles_n) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N, FM = WTM / 32, FN = WTN / 32;
  constexpr int LDH = KMAX + 8;
  constexpr int LDE = 40;
  constexpr int OPER_BYTES = (BM + BN) * LDH * 2, EPI_BYTES = (NT / 64) * 32 * LDE * 4;
  constexpr int LDS_BYTES = OPER_BYTES > EPI_BYTES ? OPER_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __bf16* const As = reinterpret_cast<__bf16*>(smem);
  __bf16* const Bs = As + BM * LDH;
  const TA* A = reinterpret_cast<const TA*>(p.A);
  TC* C = reinterpret_cast<TC*>(p.C);
  const int M = p.M, K = p.K, N = p.N;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int m_tile = tile / tiles_n;
  const int m0 = m_tile * BM;
  if (m0 >= M) return;
  const int n0 = (tile - m_tile * tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid - wm * WAVES_N;
  // A chunk: rows m0.. (lda == K), elements [m0*K, (m0+BM)*K) clamped to M*K
  {
    constexpr int EPP = 16 / sizeof(TA);        // elements per 16-byte piece
    const long base = (long)m0 * K;
    const long lim = (long)M * K;
    const int npieces = BM * K / EPP;           // K % EPP == 0
    constexpr int MAXP = BM * KMAX / EPP;
    constexpr int IT = (MAXP + NT - 1) / NT;
    typedef float f4 __attribute__((ext_vector_type(4)));
    if constexpr (sizeof(TA) == 4) {
      float4 v[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = tid + NT * it;
        long off = base + (long)e * 4;
        off = off < lim ? off : lim - 4;
        v[it] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(A) + off);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = tid + NT * it;
        if (e < npieces) {
          const int row = (e * 4) / K, k = (e * 4) - row * K;
          bf16x4 h;
          h[0] = (__bf16)v[it].x; h[1] = (__bf16)v[it].y; h[2] = (__bf16)v[it].z; h[3] = (__bf16)v[it].w;
          *reinterpret_cast<bf16x4*>(&As[row * LDH + k]) = h;
        }
      }
    } else {
      bf16x8 v[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = tid + NT * it;
        long off = base + (long)e * 8;
        off = off < lim ? off : lim - 8;
        v[it] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(A) + off);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        const int e = tid + NT * it;
        if (e < npieces) {
          const int row = (e * 8) / K, k = (e * 8) - row * K;
          *reinterpret_cast<bf16x8*>(&As[row * LDH + k]) = v[it];
        }
      }
    }
    // B tile rows n0.. [BN x K] bf16
    const int bpieces = BN * K / 8;
    constexpr int BIT = (BN * KMAX / 8 + NT - 1) / NT;
    bf16x8 w[BIT];
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
      const int e = tid + NT * it;
      int row = (e * 8) / K, k = (e * 8) - row * K;
      int gn = n0 + row;
      gn = gn < N ? gn : N - 1;
      if (e >= bpieces) { gn = n0; k = 0; }
      w[it] = *reinterpret_cast<const bf16x8*>(Bw + (long)gn * p.sbn + k);
    }
#pragma unroll
    for (int it = 0; it < BIT; ++it) {
      const int e = tid + NT * it;
      if (e < bpieces) {
        const int row = (e * 8) / K, k = (e * 8) - row * K;
        *reinterpret_cast<bf16x8*>(&Bs[row * LDH + k]) = w[it];
      }
    }
  }
  __syncthreads();
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  for (int ks = 0; ks < K / 16; ++ks) {
    bf16x8 a[FM], b[FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
    for (int j = 0; j < FN; ++j)
      b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
  __syncthreads();
  float* sE = reinterpret_cast<float*>(smem) + wid * (32 * LDE);
  const int c4 = lane & 7;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const int col = n0 + wn * WTN + j * 32 + 4 * c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = (lane >> 3) + 8 * q;
        const int row = m0 + wm * WTM + i * 32 + rl;
        float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
        if (row < M && col < N) {
          TC* dst = C + (long)row * p.ldc + col;
          if constexpr (std::is_same<TC, float>::value) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            bf16x4 h;
            h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
            *reinterpret_cast<bf16x4*>(dst) = h;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
}

// two K-steps of global loads in flight: register sets alternate, the loads of step kt + 2
// are issued while step kt computes and step kt + 1 (loaded an iteration earlier) is stored
template <int BM, int BN, int BK, int WAVES_M, int WAVES_N, typename TA, typename TC>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N) void k2(GemmParams p, const __bf16* Bw,
                                                            int tiles_n) {
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N, FM = WTM / 32, FN = WTN / 32;
  constexpr int LDH = BK + 8, GPR = BK / 8, A_G = BM * GPR, B_G = BN * GPR;
  constexpr int A_LD = (A_G + NT - 1) / NT, B_LD = (B_G + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LDH;
  constexpr int LDE = 40;
  constexpr int OPER_BYTES = 2 * STAGE * 2, EPI_BYTES = (NT / 64) * 32 * LDE * 4;
  constexpr int LDS_BYTES = OPER_BYTES > EPI_BYTES ? OPER_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __bf16* const sbase = reinterpret_cast<__bf16*>(smem);
  const TA* A = reinterpret_cast<const TA*>(p.A);
  TC* C = reinterpret_cast<TC*>(p.C);
  const int M = p.M, K = p.K, lda = p.lda, N = p.N;
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int m_tile = tile / tiles_n;
  const int m0 = m_tile * BM;
  if (m0 >= M) return;
  const int n0 = (tile - m_tile * tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid - wm * WAVES_N;
  bf16x8 ra[2][A_LD], rb[2][B_LD];
  auto gload = [&](int kt, int set) {
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      const int row = idx / GPR, k8 = idx % GPR;
      ra[set][i] = load_a8<ALOAD_DENSE, TA>(p, A, M, K, lda, m0 + (idx < A_G ? row : 0), kt * BK + 8 * k8);
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      const int n = idx / GPR, k8 = idx % GPR;
      const int gn = n0 + n, gk = kt * BK + 8 * k8;
      const int nc = gn < N ? gn : N - 1, kc = gk < K ? gk : K - 8;
      rb[set][i] = *reinterpret_cast<const bf16x8*>(Bw + (long)nc * p.sbn + kc);
    }
  };
  auto sstore = [&](int buf, int set) {
    __bf16* As = sbase + buf * STAGE;
    __bf16* Bs = As + BM * LDH;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < A_G) *reinterpret_cast<bf16x8*>(&As[(idx / GPR) * LDH + 8 * (idx % GPR)]) = ra[set][i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < B_G) *reinterpret_cast<bf16x8*>(&Bs[(idx / GPR) * LDH + 8 * (idx % GPR)]) = rb[set][i];
    }
  };
  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  auto compute = [&](int buf) {
    const __bf16* As = sbase + buf * STAGE;
    const __bf16* Bs = As + BM * LDH;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        a[i] = *reinterpret_cast<const bf16x8*>(&As[(wm * WTM + i * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
      for (int j = 0; j < FN; ++j)
        b[j] = *reinterpret_cast<const bf16x8*>(&Bs[(wn * WTN + j * 32 + (lane & 31)) * LDH + ks * 16 + 8 * (lane >> 5)]);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  };
  const int nkt = (K + BK - 1) / BK;
  gload(0, 0);
  if (nkt > 1) gload(1, 1);
  sstore(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nkt; kt += 2) {
    // even step: compute buf 0; set 0 is free -> loads of kt + 2; store set 1 (kt + 1)
    if (kt + 2 < nkt) gload(kt + 2, 0);
    compute(0);
    if (kt + 1 < nkt) sstore(1, 1);
    __syncthreads();
    if (kt + 1 >= nkt) break;
    // odd step
    if (kt + 3 < nkt) gload(kt + 3, 1);
    compute(1);
    if (kt + 2 < nkt) sstore(0, 0);
    __syncthreads();
  }
  float* sE = reinterpret_cast<float*>(smem) + wid * (32 * LDE);
  const int c4 = lane & 7;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sE[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE + (lane & 31)] = acc[i][j][r];
      __builtin_amdgcn_wave_barrier();
      const int col = n0 + wn * WTN + j * 32 + 4 * c4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rl = (lane >> 3) + 8 * q;
        const int row = m0 + wm * WTM + i * 32 + rl;
        float4 v = *reinterpret_cast<const float4*>(&sE[rl * LDE + 4 * c4]);
        if (row < M && col < N) {
          TC* dst = C + (long)row * p.ldc + col;
          if constexpr (std::is_same<TC, float>::value) {
            *reinterpret_cast<float4*>(dst) = v;
          } else {
            bf16x4 h;
            h[0] = (__bf16)v.x; h[1] = (__bf16)v.y; h[2] = (__bf16)v.z; h[3] = (__bf16)v.w;
            *reinterpret_cast<bf16x4*>(dst) = h;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
}
}  // namespace lab

struct Shape {
  const char* name;
  int M, K, N;
  bool a16, c16;
};

static double time_it(const std::function<void()>& f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  const int reps = 20;
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms * 1000.0 / reps;
}

template <typename TA, typename TC, int DBG>
static double run_lab(const GemmParams& p, const __bf16* B) {
  constexpr int BM = 128, BN = 128;
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, BM);
  return time_it([&] {
    hipLaunchKernelGGL((lab::k<BM, BN, 32, 2, 2, TA, TC, DBG>), dim3(tn * tm), dim3(256), 0, 0, p, B, tn);
  });
}

template <typename TA, typename TC>
static double run_persist(const GemmParams& p, const __bf16* B, int G) {
  constexpr int BM = 128, BN = 128;
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, BM);
  return time_it([&] {
    hipLaunchKernelGGL((lab::kp<BM, BN, 32, 2, 2, TA, TC>), dim3(G), dim3(256), 0, 0, p, B, tn, tn * tm);
  });
}

template <int BM, int BN, int BK, int WM, int WN, typename TA, typename TC>
static double run_k2(const GemmParams& p, const __bf16* B) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, BM);
  return time_it([&] {
    hipLaunchKernelGGL((lab::k2<BM, BN, BK, WM, WN, TA, TC>), dim3(tn * tm), dim3(64 * WM * WN), 0, 0, p, B, tn);
  });
}

template <int BM, int BN, int WM, int WN, typename TA, typename TC>
static double run_full(const GemmParams& p, const __bf16* B) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, BM);
  return time_it([&] {
    hipLaunchKernelGGL((lab::kf<BM, BN, 256, WM, WN, TA, TC>), dim3(tn * tm), dim3(64 * WM * WN), 0, 0, p, B, tn);
  });
}

template <typename TA, typename TC>
static void run_shape(const Shape& s, void* dA, __bf16* dB, void* dC) {
  GemmParams p{};
  p.A = reinterpret_cast<const float*>(dA);
  p.lda = s.K;
  p.sbk = 1;
  p.sbn = s.K;
  p.C = reinterpret_cast<float*>(dC);
  p.ldc = s.N;
  p.M = s.M;
  p.N = s.N;
  p.K = s.K;
  p.alpha = 1.f;
  p.max_M = s.M;
  const double bytes = (double)s.M * s.K * sizeof(TA) + (double)s.N * s.K * 2 + (double)s.M * s.N * sizeof(TC);
  const double flops = 2.0 * s.M * s.K * s.N;
  double prod = time_it([&] { launch_tile_h<32, ALOAD_DENSE, EPI_NONE, TA, TC>(p, dB, 0); });
  double full = run_lab<TA, TC, 0>(p, dB);
  double nost = run_lab<TA, TC, 1>(p, dB);
  double nomf = run_lab<TA, TC, 2>(p, dB);
  double noa = run_lab<TA, TC, 16>(p, dB);  // 16-byte bf16 epilogue stores
  double only_ld = run_lab<TA, TC, 3>(p, dB);
  double p512 = run_k2<128, 128, 32, 2, 2, TA, TC>(p, dB);
  double p768 = run_k2<128, 128, 64, 2, 2, TA, TC>(p, dB);
  double p1024 = run_k2<256, 128, 32, 4, 2, TA, TC>(p, dB);
  printf("%-8s M=%7d K=%5d N=%5d %s%s  prod %7.1f us (%5.0f GB/s %5.0f TF/s) | lab128 %7.1f  "
         "no-store %7.1f  no-mfma %7.1f  st16 %7.1f  loads-only %7.1f | pf2 128x128x32 %7.1f 128x128x64 %7.1f 256x128x32 %7.1f (best %5.0f GB/s)\n",
         s.name, s.M, s.K, s.N, s.a16 ? "A16" : "A32", s.c16 ? "C16" : "C32", prod,
         bytes / prod * 1e-3, flops / prod * 1e-6, full, nost, nomf, noa, only_ld, p512, p768, p1024,
         bytes / std::max(1e-9, std::min(p512, std::min(p768, p1024))) * 1e-3);
}

int main() {
  std::vector<Shape> shapes = {
      {"attn_in", 197370, 192, 272, false, false}, {"ff_in0", 197370, 192, 384, false, true},
      {"ff_in2", 197370, 192, 640, false, true},   {"ff_out2", 197370, 640, 192, true, false},
      {"na_in", 197370, 192, 432, false, false},   {"sa_in", 197370, 192, 48, false, true},
      {"cv_in", 197370, 192, 384, false, true},    {"cv_out", 197370, 192, 192, true, false},
      {"ff_in3", 24671, 512, 1536, false, true},   {"ff_out3", 24671, 1536, 512, true, false},
  };
  size_t maxA = 0, maxC = 0, maxB = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxB = std::max(maxB, (size_t)s.N * s.K);
  }
  void *dA, *dC;
  __bf16* dB;
  hipMalloc(&dA, maxA * 4);
  hipMalloc(&dC, maxC * 4);
  hipMalloc(&dB, maxB * 2);
  hipMemset(dA, 0, maxA * 4);
  hipMemset(dB, 0, maxB * 2);
  for (auto& s : shapes) {
    if (!s.a16 && !s.c16) run_shape<float, float>(s, dA, dB, dC);
    else if (!s.a16 && s.c16) run_shape<float, __bf16>(s, dA, dB, dC);
    else run_shape<__bf16, float>(s, dA, dB, dC);
  }
  return 0;
}
