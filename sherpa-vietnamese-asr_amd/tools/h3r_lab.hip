// gemm_h3r_kernel timing + per-wave stamps (development tool): the f16x3 mode's heaviest
// projection shapes (bench.py --shape-table), mean of 20 launches, and for block 0 the cycles
// each wave spends per tile waiting at the tile barrier, staging the A tile and in its chunks.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 [-DZASR_H3R_STAMPS] -o h3r_lab h3r_lab.hip
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

#include "../csrc/gemm_h3r.hip"

using namespace zasr;

// ffn_pack_h3_host's layout (ffn_kernels.hip): the two fp16 pieces (hi, lo 2^11), each as
// fragments [rows/16][cols/32][64 lanes][8]: element j of lane l of fragment (g, s) is
// W[16 g + (l & 15)][32 s + 8 (l >> 4) + j]
static void pack_h3(const float* w, int rows, int cols, __bf16* out) {
  const size_t n = (size_t)rows * cols;
  for (int t = 0; t < 2; ++t)
    for (int g = 0; g < rows / 16; ++g)
      for (int s = 0; s < cols / 32; ++s)
        for (int l = 0; l < 64; ++l)
          for (int j = 0; j < 8; ++j) {
            const float x = w[(size_t)(16 * g + (l & 15)) * cols + 32 * s + 8 * (l >> 4) + j];
            const _Float16 hi = (_Float16)x;
            const _Float16 v = t == 0 ? hi : (_Float16)((x - (float)hi) * 2048.f);
            std::memcpy(&out[t * n + (((size_t)g * (cols / 32) + s) * 64 + l) * 8 + j], &v, 2);
          }
}

static void run(int M, int K, int N, int epi) {
  std::mt19937 g(M + K + N);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> A((size_t)M * K), W((size_t)N * K), b(N);
  for (auto& v : A) v = nd(g);
  for (auto& v : W) v = nd(g) / std::sqrt((float)K);
  for (auto& v : b) v = 0.1f * nd(g);
  std::vector<__bf16> p(2 * W.size());
  pack_h3(W.data(), N, K, p.data());
  float *dA, *dC, *db;
  __bf16* dW;
  const int ldc = epi == EPI_GLU ? N / 2 : N;
  hipMalloc(&dA, A.size() * 4); hipMalloc(&dC, (size_t)M * ldc * 4); hipMalloc(&db, N * 4);
  hipMalloc(&dW, p.size() * 2);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dW, p.data(), p.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), N * 4, hipMemcpyHostToDevice);
  hipMemset(dC, 0, (size_t)M * ldc * 4);
  auto go = [&] { gemm_h3r(dA, dW, db, dC, ldc, M, N, K, epi, 0); };
  for (int i = 0; i < 3; ++i) go();
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i) go();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = 1000.0 * ms / 20, fl = 2.0 * M * K * N * 3;
  printf("M %d K %d N %d epi %d: %.1f us  %.3f of the fp16 peak (3 MFMA / product)\n", M, K, N, epi, us,
         fl / us / 1e6 / 2500.0);
#ifdef ZASR_H3R_STAMPS
  static long long st[8 * 64 * 4];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_h3r_stamps), sizeof(st));
  // per wave, summed over block 0's tiles: barrier wait, staging, chunks
  for (int w = 0; w < 8; ++w) {
    long long bar = 0, stg = 0, chk = 0;
    int nt = 0;
    for (int k = 0; k < 64; ++k) {
      const long long* t = st + (w * 64 + k) * 4;
      if (t[0] == 0 || t[3] < t[0]) break;
      bar += t[1] - t[0]; stg += t[2] - t[1]; chk += t[3] - t[2];
      ++nt;
    }
    printf("  wave %d: %d tiles | barrier wait %lld | A staging %lld | chunks %lld (cycles)\n", w, nt, bar, stg, chk);
  }
  std::memset(st, 0, sizeof(st));
  hipMemcpyToSymbol(HIP_SYMBOL(g_h3r_stamps), st, sizeof(st));
#endif
  fflush(stdout);
  hipFree(dA); hipFree(dC); hipFree(db); hipFree(dW);
}

int main() {
  run(49442, 384, 768, EPI_GLU);
  run(49442, 384, 384, EPI_RESADD);
  run(98813, 256, 512, EPI_GLU);
  run(49442, 384, 864, EPI_NONE);
  run(24753, 512, 1024, EPI_GLU);
  run(98813, 256, 256, EPI_RESADD);
  run(24753, 512, 512, EPI_RESADD);
  return 0;
}
