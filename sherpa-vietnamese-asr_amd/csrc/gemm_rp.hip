// Row-panel bf16 GEMM for the encoder's short-K projections (K <= 512): every projection that
// reads the f32 residual stream (attn_in, ff_in, na_in, sa_in, cv_in, encoder_proj) and the
// short-K output projections (sa_out, cv_out, na_out, residual epilogue).
//
// Why a second GEMM: at K = 48..512 the 128x128-tile kernel (gemm.hip) re-reads each A row
// panel once per N tile and pays one HBM round trip per 32-deep K slab, so a block spends
// most of its life waiting on loads it issued one slab at a time (tools/gemm_lab.hip:
// loads alone take ~45 % of its time on ff_in0).  Here one block owns BM = 64 rows and ALL N
// columns:
//   1. the whole A panel [64][K] is fetched at once (every load in flight together), rounded
//      to bf16 and parked in LDS for the life of the block -- A crosses HBM exactly once;
//   2. the block sweeps N in chunks of 128 columns, wave w computing the 64 x 32 slice of
//      column group 4c + w (two v_mfma_f32_32x32x16_bf16 per k-step sharing one B fragment);
//   3. B comes from a weight copy permuted once at load into MFMA-fragment order
//      ([N/32][K/16][64 lanes][8 bf16]): every B fragment is one fully coalesced 1 KB wave
//      load, streamed through a register ring P k-steps ahead (across chunk boundaries), so
//      the weights never touch LDS and the loop has no block barrier at all;
//   4. the epilogue stores straight from the accumulators (bias, SwooshL, residual add), bf16
//      outputs as column pairs exchanged between neighbouring lanes, and overlaps the next
//      chunk's MFMAs.
#include <type_traits>

#include "common.h"
#include "gemm.h"

namespace zasr {

namespace rp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 64;
constexpr int CHUNK = 128;  // columns per sweep step (4 waves x 32)

constexpr int round_of(int per) {  // largest divisor of per that is <= 16
  for (int r = 16; r >= 1; --r)
    if (per % r == 0 && r <= per) return r;
  return 1;
}

constexpr int ring_depth(int qk) {
  if (qk <= 8) return qk;
  for (int p = 8; p >= 2; --p)
    if (qk % p == 0) return p;
  return 1;
}

template <int EPI>
__device__ __forceinline__ float act(float v) {
  if constexpr (EPI == EPI_SWOOSHL) return swooshl_fast(v);
  if constexpr (EPI == EPI_SWOOSHR) return swooshr_fast(v);
  return v;
}

template <int K, typename TA, typename TC, int EPI>
__global__ __launch_bounds__(256) void gemm_rp_kernel(const TA* __restrict__ A, int lda,
                                                      const bf16x8* __restrict__ Bp,
                                                      const float* __restrict__ bias,
                                                      TC* __restrict__ C, int ldc, int M, int N,
                                                      int nchunks) {
  constexpr int LDK = K + 8;  // odd multiple of 16 B per row: conflict-free ds_read_b128
  constexpr int QK = K / 16;
  constexpr int P = ring_depth(QK);
  static_assert(K % 16 == 0 && QK % P == 0, "K must be a multiple of 16");
  __shared__ __attribute__((aligned(16))) __bf16 As[BM * LDK];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;
  const bf16x8* Bw = Bp + lane;

  // B ring prologue: chunk 0, k-steps 0..P-1 (in flight under the A panel fetch)
  bf16x8 ring[P];
#pragma unroll
  for (int s = 0; s < P; ++s) ring[s] = Bw[(long)(wid * QK + s) * 64];

  // A panel -> bf16 LDS image, every load of a round in flight together
  if constexpr (std::is_same<TA, float>::value) {
    constexpr int K4 = K / 4;
    constexpr int PER = BM * K4 / 256;  // = QK
    constexpr int ROUND = round_of(PER);
    static_assert(PER % ROUND == 0, "A staging rounds");
#pragma unroll
    for (int r0 = 0; r0 < PER; r0 += ROUND) {
      float4 v[ROUND];
#pragma unroll
      for (int i = 0; i < ROUND; ++i) {
        const int idx = tid + 256 * (r0 + i);
        const int row = idx / K4, k4 = idx - row * K4;
        const int gr = m0 + row < M ? m0 + row : M - 1;
        v[i] = *reinterpret_cast<const float4*>(A + (long)gr * lda + 4 * k4);
      }
#pragma unroll
      for (int i = 0; i < ROUND; ++i) {
        const int idx = tid + 256 * (r0 + i);
        const int row = idx / K4, k4 = idx - row * K4;
        bf16x4 hv;
        hv[0] = (__bf16)v[i].x;
        hv[1] = (__bf16)v[i].y;
        hv[2] = (__bf16)v[i].z;
        hv[3] = (__bf16)v[i].w;
        *reinterpret_cast<bf16x4*>(&As[row * LDK + 4 * k4]) = hv;
      }
    }
  } else {
    constexpr int K8 = K / 8;
    constexpr int PIECES = BM * K8;
    constexpr int PER = (PIECES + 255) / 256;
    constexpr int ROUND = round_of(PER);
    static_assert(PER % ROUND == 0, "A staging rounds");
#pragma unroll
    for (int r0 = 0; r0 < PER; r0 += ROUND) {
      bf16x8 v[ROUND];
#pragma unroll
      for (int i = 0; i < ROUND; ++i) {
        const int idx0 = tid + 256 * (r0 + i);
        const int idx = idx0 < PIECES ? idx0 : PIECES - 1;
        const int row = idx / K8, k8 = idx - row * K8;
        const int gr = m0 + row < M ? m0 + row : M - 1;
        v[i] = *reinterpret_cast<const bf16x8*>(A + (long)gr * lda + 8 * k8);
      }
#pragma unroll
      for (int i = 0; i < ROUND; ++i) {
        const int idx = tid + 256 * (r0 + i);
        if (PIECES % 256 == 0 || idx < PIECES) {
          const int row = idx / K8, k8 = idx - row * K8;
          *reinterpret_cast<bf16x8*>(&As[row * LDK + 8 * k8]) = v[i];
        }
      }
    }
  }
  __syncthreads();

  const int r32 = lane & 31, h = lane >> 5;
  const __bf16* a0p = &As[r32 * LDK + 8 * h];
  const __bf16* a1p = &As[(32 + r32) * LDK + 8 * h];
  for (int c = 0; c < nchunks; ++c) {
    const int g = c * 4 + wid;
    f32x16 acc0, acc1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc0[r] = 0.f;
      acc1[r] = 0.f;
    }
#pragma unroll
    for (int q = 0; q < QK; ++q) {
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(a0p + 16 * q);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(a1p + 16 * q);
      const bf16x8 b = ring[q % P];
      acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, b, acc1, 0, 0, 0);
      // refill this slot with the k-step P ahead (next chunk's first steps at the tail)
      if (q + P < QK) {
        ring[q % P] = Bw[(long)(g * QK + q + P) * 64];
      } else if (c + 1 < nchunks) {
        ring[q % P] = Bw[(long)((g + 4) * QK + q + P - QK) * 64];
      }
    }

    // epilogue straight from the accumulators: lane = column r32, rows (r&3) + 8(r>>2) + 4h
    const int col = g * 32 + r32;
    const bool cv = col < N;
    const float bc = (bias != nullptr && cv) ? bias[col] : 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x16& acc = t ? acc1 : acc0;
      const int rb = m0 + 32 * t + 4 * h;
      if constexpr (std::is_same<TC, float>::value) {
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = act<EPI>(acc[r] + bc);
        if constexpr (EPI == EPI_RESADD) {
          float o[16];
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = rb + (r & 3) + 8 * (r >> 2);
            const int rr = row < M ? row : M - 1;
            o[r] = C[(long)rr * ldc + (cv ? col : N - 1)];  // unconditional (clamped) load
          }
#pragma unroll
          for (int r = 0; r < 16; ++r) v[r] += o[r];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rb + (r & 3) + 8 * (r >> 2);
          if (cv && row < M) C[(long)row * ldc + col] = v[r];
        }
      } else {
        // column pairs: even lane stores (row_r, col..col+1), odd lane (row_r+1, col-1..col)
        const bool odd = (lane & 1) != 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float e = act<EPI>(acc[2 * i] + bc);
          const float o = act<EPI>(acc[2 * i + 1] + bc);
          const float x = __shfl_xor(odd ? e : o, 1, 64);
          bf16x2 pr;
          pr[0] = (__bf16)(odd ? x : e);
          pr[1] = (__bf16)(odd ? o : x);
          const int r = 2 * i + (odd ? 1 : 0);
          const int row = rb + (r & 3) + 8 * (r >> 2);
          const int cc = odd ? col - 1 : col;
          if (cc < N && row < M) *reinterpret_cast<bf16x2*>(C + (long)row * ldc + cc) = pr;
        }
      }
    }
  }
}

// Bp[g][q][lane][j] = W[32g + (lane & 31)][16q + 8(lane >> 5) + j], zero beyond N
__global__ void permute_rp_kernel(const __bf16* __restrict__ W, int N, int K, int ngroups,
                                  bf16x8* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int QK = K / 16;
  if (i >= (long)ngroups * QK * 64) return;
  const int lane = (int)(i & 63);
  const long gq = i >> 6;
  const int g = (int)(gq / QK), q = (int)(gq - (long)g * QK);
  const int n = 32 * g + (lane & 31);
  const int k = 16 * q + 8 * (lane >> 5);
  bf16x8 v;
  if (n < N) {
    v = *reinterpret_cast<const bf16x8*>(W + (long)n * K + k);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)0.f;
  }
  out[i] = v;
}

template <int K, typename TA, typename TC, int EPI>
void launch(const void* A, int lda, const void* Bp, const float* bias, void* C, int ldc, int M,
            int N, hipStream_t st) {
  const int nchunks = cdiv(N, CHUNK);
  ZASR_LAUNCH((gemm_rp_kernel<K, TA, TC, EPI>), dim3(cdiv(M, BM)), dim3(256), 0, st,
                     reinterpret_cast<const TA*>(A), lda, reinterpret_cast<const bf16x8*>(Bp),
                     bias, reinterpret_cast<TC*>(C), ldc, M, N, nchunks);
}

// combinations the encoder uses: (a_bf16, c_bf16, epi)
template <int K>
bool dispatch_k(const void* A, bool a16, int lda, const void* Bp, const float* bias, void* C,
                bool c16, int ldc, int M, int N, int epi, hipStream_t st) {
  if (!a16 && c16 && epi == EPI_NONE) {
    launch<K, float, __bf16, EPI_NONE>(A, lda, Bp, bias, C, ldc, M, N, st);
  } else if (!a16 && c16 && epi == EPI_SWOOSHL) {
    launch<K, float, __bf16, EPI_SWOOSHL>(A, lda, Bp, bias, C, ldc, M, N, st);
  } else if (!a16 && !c16 && epi == EPI_NONE) {
    launch<K, float, float, EPI_NONE>(A, lda, Bp, bias, C, ldc, M, N, st);
  } else if (a16 && !c16 && epi == EPI_RESADD) {
    launch<K, __bf16, float, EPI_RESADD>(A, lda, Bp, bias, C, ldc, M, N, st);
  } else {
    return false;
  }
  return true;
}

}  // namespace rp

bool gemm_rp_supported_k(int K) {
  switch (K) {
    case 48: case 64: case 96: case 128: case 144: case 192: case 256: case 288: case 384:
    case 512:
      return true;
    default:
      return false;
  }
}

long gemm_rp_packed_elems(int N, int K) { return (long)cdiv(N, rp::CHUNK) * rp::CHUNK * K; }

void gemm_rp_pack_weights(const void* W, int N, int K, void* out, hipStream_t st) {
  ZASR_REQUIRE(K % 16 == 0, "gemm_rp: K must be a multiple of 16");
  const int ngroups = cdiv(N, rp::CHUNK) * (rp::CHUNK / 32);
  const long n = (long)ngroups * (K / 16) * 64;
  ZASR_LAUNCH(rp::permute_rp_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st,
                     reinterpret_cast<const __bf16*>(W), N, K, ngroups,
                     reinterpret_cast<rp::bf16x8*>(out));
}

bool gemm_rp(const void* A, bool a_bf16, int lda, const void* Bp, const float* bias, void* C,
             bool c_bf16, int ldc, int M, int N, int K, int epi, hipStream_t st) {
  if (M <= 0) return true;
  if (N % 4 != 0 || (a_bf16 ? lda % 8 : lda % 4) != 0 || ldc % 2 != 0) return false;
  switch (K) {
#define ZASR_RP_K(k) \
  case k: return rp::dispatch_k<k>(A, a_bf16, lda, Bp, bias, C, c_bf16, ldc, M, N, epi, st);
    ZASR_RP_K(48) ZASR_RP_K(64) ZASR_RP_K(96) ZASR_RP_K(128) ZASR_RP_K(144) ZASR_RP_K(192)
    ZASR_RP_K(256) ZASR_RP_K(288) ZASR_RP_K(384) ZASR_RP_K(512)
#undef ZASR_RP_K
    default:
      return false;
  }
}

}  // namespace zasr
