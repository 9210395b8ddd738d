// f16x3 GEMM lab (development tool, not part of libzasr): a one-accumulator 8-wave kernel
// (gemm_h3p_kernel, below; measured slower than the library's kernel on every shape but one,
// profiles/r05/h3p_lab.txt) against the default LDS-DMA kernel (gemm_glds_h3_kernel, read-before-
// issue, 4 x 1 waves) on the heaviest f16x3 projection shapes of the 68M bench step.  Per
// variant: mean of 10 launches after 2 warm-ups, the max error of 512 sampled outputs against
// an f64 host reference (relative to sum |a||w| + |b| of the output), and the largest
// difference from the default kernel's output relative to that magnitude.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o h3p_lab h3p_lab.hip
#include "../csrc/gemm_x3.hip"

namespace zasr {
namespace {
// ---------------------------------------------------------------------------------------
// f16x3, one accumulator, one block of 8 waves per CU ("h3p"): a 256-row tile with the
// products on ONE scale, so each output fragment needs one accumulator instead of two:
//   acc += a_lo * w_hi + a_hi * w_lo + a_hi * (w_hi * 2^11)      = 2^11 * a w (lo * lo dropped)
// (w_hi * 2^11 is exact in fp16 for |w| < 32, checked at load: gemm_h3p_ok), scaled by 2^-11
// in the epilogue.  The freed accumulators pay for a 64 x 128 wave tile (8 waves as 4 x 2,
// block tile 256 x 256): per k-step a wave reads 2 A fragments (f32, split in registers) and
// 4 x 2 W piece fragments for 24 MFMAs, twice the MFMAs per operand byte of the 128 x 128
// kernel above.  Pipeline: NS LDS stages filled by global_load_lds, counted vmcnt + raw
// s_barrier (never vmcnt(0) in the loop), the fragment reads as inline-asm ds_read_b128 so the
// compiler does not drain the DMA in flight before them (it cannot tell the stages apart), the
// next stage's DMA issued right after the barrier, MFMA clusters at raised priority.
// ---------------------------------------------------------------------------------------
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  typedef const __attribute__((address_space(3))) unsigned char* lds_cptr;
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((lds_cptr)p));
}
__device__ __forceinline__ u32x4 ds_read16(unsigned addr) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr) : "memory");
  return r;
}

// f16x3 epilogue with one accumulator on the 2^11 scale (h3_epilogue's layout and epilogues)
template <int EPI, int FM, int FN>
__device__ __forceinline__ void h3p_epilogue(const GemmParams& p, float* sE,
                                             const f32x16 (&acc)[FM][FN], int row0, int col0,
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
        sE[((r & 3) + 8 * (r >> 2) + 4 * h) * LDE + r32] = acc[i][j][r] * kF16LoInv;
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
          if constexpr (EPI == EPI_GLU) {
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

template <int NS, int EPI, int BN, int WM>
__global__ __launch_bounds__(512, 1) void gemm_h3p_kernel(GemmParams p, const __bf16* Bw, long blo,
                                                         int tiles_n) {
  constexpr int BM = 256, BK = 32, NW = 8;
  constexpr int WN = NW / WM;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 4;       // f32 rows of 128 B
  constexpr int B_BYTES = BN * BK * 2;       // one fp16 piece, rows of 64 B
  constexpr int STAGE = A_BYTES + 2 * B_BYTES;
  constexpr int GA = A_BYTES / 1024 / NW;    // 1 KB DMA pieces per wave
  constexpr int GB = B_BYTES / 1024 / NW;
  constexpr int G = GA + 2 * GB;
  constexpr int LDE = 40;
  constexpr int EPI_BYTES = NW * 32 * LDE * 4;
  constexpr int LDS_BYTES = NS * STAGE > EPI_BYTES ? NS * STAGE : EPI_BYTES;
  static_assert(NS >= 2 && NS <= 3 && LDS_BYTES <= 160 * 1024, "stages / LDS");
  static_assert(GA >= 1 && GB >= 1 && FM >= 1 && FN >= 1, "tile");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[LDS_BYTES];

  const int lin = xcd_tile(blockIdx.x, gridDim.x);
  const int m_tile = lin / tiles_n;
  const int m0 = m_tile * BM, n0 = (lin - m_tile * tiles_n) * BN;
  const float* A = p.A;
  const int M = p.M, K = p.K, lda = p.lda, N = p.N;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int nkt = K / BK;

  const float* asrc[GA];
  const __bf16* bsrc[GB];
#pragma unroll
  for (int g = 0; g < GA; ++g) {
    const int row = (wid * GA + g) * 8 + (lane >> 3);
    const int lc = (lane & 7) ^ ((row >> 1) & 7);
    const int gr = m0 + row < M ? m0 + row : M - 1;
    asrc[g] = A + (long)gr * lda + 4 * lc;
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
#pragma unroll
    for (int g = 0; g < GA; ++g)
      __builtin_amdgcn_global_load_lds(const_cast<float*>(asrc[g] + k0),
                                       (h3_lds_t)(st + (wid * GA + g) * 1024), 16, 0, 0);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < GB; ++g)
        __builtin_amdgcn_global_load_lds(const_cast<__bf16*>(bsrc[g] + t * blo + k0),
                                         (h3_lds_t)(st + A_BYTES + t * B_BYTES + (wid * GB + g) * 1024),
                                         16, 0, 0);
  };

  f32x16 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkt) issue(s);
  const int r32 = lane & 31, h = lane >> 5;
  const unsigned base = lds_addr(smem);
  // per-lane LDS byte offsets within a stage of this wave's fragment rows (k-step chunk ch
  // applied below): A row = wm * WTM + i * 32 + r32, B row = wn * WTN + j * 32 + r32
  unsigned aoff[FM][4], boff[FN][2];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int row = wm * WTM + i * 32 + r32;
    const int sw = (row >> 1) & 7;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + h;
      aoff[i][2 * ks] = row * 128 + (((2 * ch) ^ sw) << 4);
      aoff[i][2 * ks + 1] = row * 128 + (((2 * ch + 1) ^ sw) << 4);
    }
  }
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int row = wn * WTN + j * 32 + r32;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) boff[j][ks] = A_BYTES + row * 64 + (((2 * ks + h) ^ ((row >> 2) & 3)) << 4);
  }
  for (int kt = 0; kt < nkt; ++kt) {
    // stage kt landed (this wave's pieces; the barrier makes it every wave's) with the stages
    // after it still in flight; at the tail fewer stages remain outstanding
    if constexpr (NS == 3) {
      if (kt + 1 < nkt) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    // every wave finished reading stage kt - 1 (its reads were waited for before its MFMAs):
    // refill it with stage kt + NS - 1
    if (kt + NS - 1 < nkt) issue(kt + NS - 1);
    const unsigned st = base + (kt % NS) * STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      u32x4 ra[FM][2], rb[FN][2];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        ra[i][0] = ds_read16(st + aoff[i][2 * ks]);
        ra[i][1] = ds_read16(st + aoff[i][2 * ks + 1]);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        rb[j][0] = ds_read16(st + boff[j][ks]);
        rb[j][1] = ds_read16(st + boff[j][ks] + B_BYTES);
      }
      // the reads' results exist for the compiler only after this wait (each fragment an
      // in-out operand of an asm statement behind it)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < FM; ++i) asm volatile("" : "+v"(ra[i][0]), "+v"(ra[i][1]));
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" : "+v"(rb[j][0]), "+v"(rb[j][1]));
      f16x8 ah[FM], al[FM], bh[FN], bl[FN], bs[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const float4 x0 = __builtin_bit_cast(float4, ra[i][0]);
        const float4 x1 = __builtin_bit_cast(float4, ra[i][1]);
        const float v[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          ah[i][q] = (_Float16)v[q];
          al[i][q] = (_Float16)((v[q] - (float)ah[i][q]) * kF16Lo);
        }
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        bh[j] = __builtin_bit_cast(f16x8, rb[j][0]);
        bl[j] = __builtin_bit_cast(f16x8, rb[j][1]);
        bs[j] = bh[j] * (_Float16)kF16Lo;  // exact: |w_hi| < 32 (gemm_h3p_ok)
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[i], bs[j], acc[i][j], 0, 0, 0);
        }
      __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  h3p_epilogue<EPI, FM, FN>(p, reinterpret_cast<float*>(smem) + wid * (32 * LDE), acc,
                            m0 + wm * WTM, n0 + wn * WTN, lane);
}

template <int NS, int EPI, int BN, int WM>
void launch_h3p(const GemmParams& p, const __bf16* Bw, long blo, hipStream_t st) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, 256);
  hipLaunchKernelGGL((gemm_h3p_kernel<NS, EPI, BN, WM>), dim3(tn * tm), dim3(512), 0, st, p, Bw,
                     blo, tn);
}

}  // namespace
}  // namespace zasr

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  const char* name;
  int M, K, N;
};

typedef void (*LaunchFn)(const GemmParams&, const __bf16*, long, hipStream_t);
struct V {
  const char* name;
  int bn;
  LaunchFn fn;
};

int main(int argc, char** argv) {
  const Shape shapes[] = {
      {"qkp d384", 49442, 384, 768},     {"ffn_in d384", 49442, 384, 1280},
      {"ffn_out d384", 49442, 1280, 384}, {"ffn_in d256", 98813, 256, 960},
      {"ffn_out d256", 98813, 960, 256},  {"ffn_in d512", 24753, 512, 1920},
      {"ffn_in d192", 197561, 192, 768},  {"ffn_out d192", 197561, 768, 192},
  };
  const V vars[] = {
      {"default glds rb 128", 128, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_glds_h3<2, EPI_NONE, 128, 4, 3, ALOAD_DENSE, 1>(q, b, lo, st); }},
      {"default glds rb 64", 64, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_glds_h3<2, EPI_NONE, 64, 4, 3, ALOAD_DENSE, 1>(q, b, lo, st); }},
      {"h3p ns2 bn256 4x2", 256, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_h3p<2, EPI_NONE, 256, 4>(q, b, lo, st); }},
      {"h3p ns3 bn128 4x2", 128, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_h3p<3, EPI_NONE, 128, 4>(q, b, lo, st); }},
      {"h3p ns3 bn128 8x1", 128, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_h3p<3, EPI_NONE, 128, 8>(q, b, lo, st); }},
      {"h3p ns2 bn128 4x2", 128, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
         launch_h3p<2, EPI_NONE, 128, 4>(q, b, lo, st); }},
  };
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  uint32_t st = 12345u;
  auto nd = [&]() {  // uniform in [-1.7, 1.7) (unit variance)
    st = st * 1664525u + 1013904223u;
    return ((st >> 8) * (1.0f / 16777216.0f) - 0.5f) * 3.4641f;
  };
  for (int si = 0; si < (int)(sizeof(shapes) / sizeof(shapes[0])); ++si) {
    if (only >= 0 && si != only) continue;
    const Shape& s = shapes[si];
    const size_t na = (size_t)s.M * s.K, nw = (size_t)s.N * s.K, nc = (size_t)s.M * s.N;
    std::vector<float> hA(na), hW(nw), hb(s.N);
    for (auto& x : hA) x = nd();
    const float ws = 1.f / std::sqrt((float)s.K);
    for (auto& x : hW) x = nd() * ws;
    for (auto& x : hb) x = 0.1f * nd();
    float *dA, *dW, *db, *dC;
    __bf16* dWx;
    hipMalloc(&dA, na * 4);
    hipMalloc(&dW, nw * 4);
    hipMalloc(&dWx, nw * 2 * 2);
    hipMalloc(&db, s.N * 4);
    hipMalloc(&dC, nc * 4);
    hipMemcpy(dA, hA.data(), na * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW, hW.data(), nw * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), s.N * 4, hipMemcpyHostToDevice);
    split_to_bf16(dW, dWx, (long)nw, kPiecesF16, 0);
    GemmParams p{};
    p.A = dA;
    p.lda = s.K;
    p.B = dW;
    p.sbk = 1;
    p.sbn = s.K;
    p.C = dC;
    p.ldc = s.N;
    p.bias = db;
    p.M = s.M;
    p.N = s.N;
    p.K = s.K;
    p.alpha = 1.f;
    p.max_M = s.M;
    std::mt19937 r2(11);
    std::vector<long> sm(512), sn(512);
    std::vector<double> ref(512), mag(512);
    for (int t = 0; t < 512; ++t) {
      sm[t] = r2() % s.M;
      sn[t] = r2() % s.N;
      double acc = hb[sn[t]], mg = std::fabs(hb[sn[t]]);
      for (int k = 0; k < s.K; ++k) {
        acc += (double)hA[sm[t] * s.K + k] * hW[sn[t] * s.K + k];
        mg += std::fabs((double)hA[sm[t] * s.K + k] * hW[sn[t] * s.K + k]);
      }
      ref[t] = acc;
      mag[t] = mg;
    }
    std::vector<float> first;
    for (const V& v : vars) {
      if (s.N % 4) continue;
      hipMemset(dC, 0, nc * 4);
      v.fn(p, dWx, (long)nw, 0);
      if (hipDeviceSynchronize() != hipSuccess) {
        printf("%s: launch failed\n", v.name);
        return 1;
      }
      std::vector<float> got(nc);
      hipMemcpy(got.data(), dC, nc * 4, hipMemcpyDeviceToHost);
      double emax = 0.0, dmax = 0.0;
      for (int t = 0; t < 512; ++t) {
        const double g = got[sm[t] * s.N + sn[t]];
        emax = std::max(emax, std::fabs(g - ref[t]) / mag[t]);
        if (!first.empty()) dmax = std::max(dmax, std::fabs(g - first[sm[t] * s.N + sn[t]]) / mag[t]);
      }
      if (first.empty()) first = got;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int w = 0; w < 2; ++w) v.fn(p, dWx, (long)nw, 0);
      hipEventRecord(e0, 0);
      for (int it = 0; it < 10; ++it) v.fn(p, dWx, (long)nw, 0);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      const double f32flops = 2.0 * s.M * s.K * s.N;
      printf("%-13s %-20s %8.1f us  fp16 mfma %.3f of 2.5 PF  err %.2e  vs_default %.2e\n", s.name,
             v.name, us, 3 * f32flops / us * 1e-6 / 2500.0, emax, dmax);
      fflush(stdout);
    }
    hipFree(dA); hipFree(dW); hipFree(dWx); hipFree(db); hipFree(dC);
  }
  return 0;
}
