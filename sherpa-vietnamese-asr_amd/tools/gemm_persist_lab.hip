// Persistent tile loop for the f32-A -> bf16-C encoder in-projections (development lab, not
// part of libzasr).  gemm_bf16_kernel's DEEP path (two register sets of
// 32-deep slabs) with the grid sized to the resident blocks: each block walks a strided range
// of its XCD's contiguous tile range, and the loads of the NEXT tile's slabs 0 / 1 go out in
// place of the clamped tail loads of the current tile, so they are in flight while the
// current tile's epilogue transposes and stores (bias preloaded at tile start: the epilogue
// issues no global load that would wait behind them).  Same slabs, same MFMA order, same
// epilogue arithmetic: outputs bit-identical to launch_h (checked on sampled outputs).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o gemm_persist_lab gemm_persist_lab.hip
#include "../csrc/gemm.hip"

#include <cstdio>
#include <random>
#include <vector>

using namespace zasr;

template <int BM, int BN, int WAVES_M, int WAVES_N>
__global__ __launch_bounds__(64 * WAVES_M* WAVES_N)
__attribute__((amdgpu_waves_per_eu(WAVES_M * WAVES_N >= 8 ? 4 : 2))) void gemm_persist_kernel(
    GemmParams p, const __bf16* Bw, int tiles_n, int tiles_m) {
  constexpr int BK = 32;
  constexpr int NT = 64 * WAVES_M * WAVES_N;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int FM = WTM / 32, FN = WTN / 32;
  static_assert(FN % 2 == 0, "paired epilogue");
  constexpr int LDH = BK + 8, GPR = BK / 8;
  constexpr int A_G = BM * GPR, B_G = BN * GPR;
  constexpr int A_LD = (A_G + NT - 1) / NT, B_LD = (B_G + NT - 1) / NT;
  constexpr int STAGE = (BM + BN) * LDH;
  constexpr int LDE2 = 72;
  constexpr int OPER_BYTES = 2 * STAGE * 2;
  constexpr int EPI_BYTES = (NT / 64) * 32 * LDE2 * 4;
  constexpr int LDS_BYTES = OPER_BYTES > EPI_BYTES ? OPER_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) unsigned char smem[LDS_BYTES];
  __bf16* const sbase = reinterpret_cast<__bf16*>(smem);

  const float* A = p.A;
  __bf16* C = reinterpret_cast<__bf16*>(p.C);
  const int M = p.M, K = p.K, N = p.N, lda = p.lda;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WAVES_N, wn = wid - wm * WAVES_N;
  const int nkt = K / BK;
  // XCD x (= block % 8) owns tiles [T x / 8, T (x + 1) / 8) in row-panel order; its GS blocks
  // take every GS-th tile of that range
  const int T = tiles_n * tiles_m;
  const int x = blockIdx.x & 7, GS = gridDim.x >> 3;
  const int t_end = (int)((long)T * (x + 1) / 8);
  int tile = (int)((long)T * x / 8) + (blockIdx.x >> 3);
  if (tile >= t_end) return;

  const float* arow[A_LD];
  const __bf16* brow[B_LD];
  auto ptrs = [&](int t, const float* (&ar)[A_LD], const __bf16* (&br)[B_LD]) {
    const int mt = t / tiles_n;
    const int m0 = mt * BM, n0 = (t - mt * tiles_n) * BN;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      const int row = (idx < A_G ? idx : 0) / GPR, k8 = idx % GPR;
      const int gm = m0 + row < M ? m0 + row : M - 1;
      ar[i] = A + (long)gm * lda + 8 * k8;
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      const int n = (idx < B_G ? idx : 0) / GPR, k8 = idx % GPR;
      const int gn = n0 + n < N ? n0 + n : N - 1;
      br[i] = Bw + (long)gn * p.sbn + 8 * k8;
    }
  };
  auto to_bf16x8 = [](float4 x0, float4 x1) {
    bf16x8 v;
    v[0] = (__bf16)x0.x; v[1] = (__bf16)x0.y; v[2] = (__bf16)x0.z; v[3] = (__bf16)x0.w;
    v[4] = (__bf16)x1.x; v[5] = (__bf16)x1.y; v[6] = (__bf16)x1.z; v[7] = (__bf16)x1.w;
    return v;
  };
  bf16x8 xa[2][A_LD], xb[2][B_LD];
  auto gl = [&](bf16x8 (&ra_)[A_LD], bf16x8 (&rb_)[B_LD], const float* const (&ar)[A_LD],
                const __bf16* const (&br)[B_LD], int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const float* a = ar[i] + k0;
      ra_[i] = to_bf16x8(*reinterpret_cast<const float4*>(a), *reinterpret_cast<const float4*>(a + 4));
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) rb_[i] = *reinterpret_cast<const bf16x8*>(br[i] + k0);
  };
  auto ss = [&](const bf16x8 (&ra_)[A_LD], const bf16x8 (&rb_)[B_LD], int buf) {
    __bf16* As = sbase + buf * STAGE;
    __bf16* Bs = As + BM * LDH;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < A_G) *reinterpret_cast<bf16x8*>(&As[(idx / GPR) * LDH + 8 * (idx % GPR)]) = ra_[i];
    }
#pragma unroll
    for (int i = 0; i < B_LD; ++i) {
      const int idx = tid + NT * i;
      if (idx < B_G) *reinterpret_cast<bf16x8*>(&Bs[(idx / GPR) * LDH + 8 * (idx % GPR)]) = rb_[i];
    }
  };
  auto bar = []() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  f32x16 acc[FM][FN];
  auto mma_slab = [&](int cur) {
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
  };

  ptrs(tile, arow, brow);
  gl(xa[0], xb[0], arow, brow, 0);
  gl(xa[1], xb[1], arow, brow, 1);
  while (true) {
    const int mt = tile / tiles_n;
    const int m0 = mt * BM, n0 = (tile - mt * tiles_n) * BN;
    const int next = tile + GS;
    const bool has_next = next < t_end;
    const float* narow[A_LD];
    const __bf16* nbrow[B_LD];
    ptrs(has_next ? next : tile, narow, nbrow);
    // this tile's bias columns, loaded before the next tile's slabs are issued
    const int c8 = lane & 7;
    float4 bias[FN / 2][2];
#pragma unroll
    for (int j = 0; j < FN; j += 2) {
      const int col = n0 + wn * WTN + j * 32 + 8 * c8;
      bias[j / 2][0] = bias[j / 2][1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (p.bias && col < N) {
        bias[j / 2][0] = *reinterpret_cast<const float4*>(p.bias + col);
        bias[j / 2][1] = *reinterpret_cast<const float4*>(p.bias + col + 4);
      }
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    ss(xa[0], xb[0], 0);
    bar();
    for (int kt = 0; kt < nkt; kt += 2) {
      // slab kt + 2 / kt + 3 of this tile, or (past its end) slab 0 / 1 of the next one
      if (kt + 2 < nkt) gl(xa[0], xb[0], arow, brow, kt + 2);
      else gl(xa[0], xb[0], narow, nbrow, kt + 2 - nkt);
      mma_slab(0);
      ss(xa[1], xb[1], 1);
      bar();
      if (kt + 3 < nkt) gl(xa[1], xb[1], arow, brow, kt + 3);
      else gl(xa[1], xb[1], narow, nbrow, kt + 3 - nkt);
      mma_slab(1);
      if (kt + 2 < nkt) {
        ss(xa[0], xb[0], 0);
        bar();
      }
    }
    bar();  // LDS-only (no vmcnt wait: the next tile's slabs stay in flight); the epilogue reuses the operand buffers
    float* sP = reinterpret_cast<float*>(smem) + wid * (32 * LDE2);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int j = 0; j < FN; j += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            sP[((r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * LDE2 + 32 * h + (lane & 31)] = acc[i][j + h][r];
        __builtin_amdgcn_wave_barrier();
        const int col = n0 + wn * WTN + j * 32 + 8 * c8;
        const float4 b0 = bias[j / 2][0], b1 = bias[j / 2][1];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rl = (lane >> 3) + 8 * q;
          const int row = m0 + wm * WTM + i * 32 + rl;
          const float4 v0 = *reinterpret_cast<const float4*>(&sP[rl * LDE2 + 8 * c8]);
          const float4 v1 = *reinterpret_cast<const float4*>(&sP[rl * LDE2 + 8 * c8 + 4]);
          if (row < M && col < N) {
            bf16x8 hv;
            hv[0] = (__bf16)fmaf(v0.x, p.alpha, b0.x);
            hv[1] = (__bf16)fmaf(v0.y, p.alpha, b0.y);
            hv[2] = (__bf16)fmaf(v0.z, p.alpha, b0.z);
            hv[3] = (__bf16)fmaf(v0.w, p.alpha, b0.w);
            hv[4] = (__bf16)fmaf(v1.x, p.alpha, b1.x);
            hv[5] = (__bf16)fmaf(v1.y, p.alpha, b1.y);
            hv[6] = (__bf16)fmaf(v1.z, p.alpha, b1.z);
            hv[7] = (__bf16)fmaf(v1.w, p.alpha, b1.w);
            *reinterpret_cast<bf16x8*>(C + (long)row * p.ldc + col) = hv;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    if (!has_next) break;
    bar();  // every wave's epilogue reads are done before buffer 0 is refilled
    tile = next;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) arow[i] = narow[i];
#pragma unroll
    for (int i = 0; i < B_LD; ++i) brow[i] = nbrow[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int BM, int BN, int WM, int WN>
static void launch_persist(const GemmParams& p, const __bf16* Bw, int grid) {
  const int tn = cdiv(p.N, BN), tm = cdiv(p.M, BM);
  hipLaunchKernelGGL((gemm_persist_kernel<BM, BN, WM, WN>), dim3(grid), dim3(64 * WM * WN), 0, 0, p,
                     Bw, tn, tm);
}

struct Shape {
  int M, K, N;
};

int main() {
  // the f32-A -> bf16-C in-projections of the 68M bench step with K % 64 == 0
  std::vector<Shape> shapes = {{49442, 384, 768}, {98813, 256, 512}, {49442, 384, 864},
                               {24753, 512, 1024}, {98813, 256, 576}, {24753, 512, 1152},
                               {98813, 256, 272}, {24753, 512, 544}};
  size_t maxA = 0, maxC = 0, maxB = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxB = std::max(maxB, (size_t)s.N * s.K);
  }
  float *dA, *dbias;
  __bf16 *dB, *dC, *dRef;
  (void)hipMalloc(&dA, maxA * 4);
  (void)hipMalloc(&dB, maxB * 2);
  (void)hipMalloc(&dC, maxC * 2);
  (void)hipMalloc(&dRef, maxC * 2);
  (void)hipMalloc(&dbias, 4096 * 4);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> hA(maxA), hbias(4096);
  std::vector<__bf16> hB(maxB);
  for (auto& v : hA) v = nd(rng);
  for (auto& v : hB) v = (__bf16)(nd(rng) * 0.08f);
  for (auto& v : hbias) v = nd(rng) * 0.1f;
  (void)hipMemcpy(dA, hA.data(), maxA * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB.data(), maxB * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(dbias, hbias.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](auto fn) {
    fn();
    fn();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) fn();
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms * 100.f;  // us per launch
  };
  auto same = [&](size_t n) {
    std::mt19937 r2(11);
    for (int q = 0; q < 2048; ++q) {
      const size_t idx = (size_t)r2() % n;
      unsigned short a = 0, b = 0;
      (void)hipMemcpy(&a, dC + idx, 2, hipMemcpyDeviceToHost);
      (void)hipMemcpy(&b, dRef + idx, 2, hipMemcpyDeviceToHost);
      if (a != b) return false;
    }
    return true;
  };
  for (auto& s : shapes) {
    GemmParams p{};
    p.A = dA;
    p.lda = s.K;
    p.sbk = 1;
    p.sbn = s.K;
    p.C = reinterpret_cast<float*>(dRef);
    p.ldc = s.N;
    p.bias = dbias;
    p.M = s.M;
    p.N = s.N;
    p.K = s.K;
    p.alpha = 1.f;
    p.max_M = s.M;
    launch_h<128, 128, 32, 2, 2, ALOAD_DENSE, EPI_NONE, float, __bf16>(p, dB, 0);
    const float t128 = time([&] { launch_h<128, 128, 32, 2, 2, ALOAD_DENSE, EPI_NONE, float, __bf16>(p, dB, 0); });
    const float t256 = time([&] { launch_h<128, 256, 32, 2, 4, ALOAD_DENSE, EPI_NONE, float, __bf16>(p, dB, 0); });
    printf("M=%6d K=%4d N=%5d: 128x128 %.1f  128x256 %.1f |", s.M, s.K, s.N, t128, t256);
    p.C = reinterpret_cast<float*>(dC);
    for (int g : {256, 512, 768, 1024}) {
      (void)hipMemset(dC, 0, (size_t)s.M * s.N * 2);
      launch_persist<128, 128, 2, 2>(p, dB, g);
      (void)hipDeviceSynchronize();
      const bool ok = same((size_t)s.M * s.N);
      const float t = time([&] { launch_persist<128, 128, 2, 2>(p, dB, g); });
      printf("  p128x128/g%d %.1f%s", g, t, ok ? "" : "(DIFF)");
    }
    for (int g : {256, 512}) {
      (void)hipMemset(dC, 0, (size_t)s.M * s.N * 2);
      launch_persist<128, 256, 2, 4>(p, dB, g);
      (void)hipDeviceSynchronize();
      const bool ok = same((size_t)s.M * s.N);
      const float t = time([&] { launch_persist<128, 256, 2, 4>(p, dB, g); });
      printf("  p128x256/g%d %.1f%s", g, t, ok ? "" : "(DIFF)");
    }
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
