// Split-product GEMM lab (development tool, not part of libzasr): the bf16x6 (3 bf16 pieces,
// 6 MFMAs) and f16x3 (2 fp16 pieces hi + lo * 2^-11, 3 MFMAs, two accumulators) formats of
// gemm_x3 on the heaviest encoder projection shapes of the 68M bench step, through the
// library entry point gemm_x3(); mean of 10 launches after 2 warm-ups, and the max error of
// 512 sampled outputs against an f64 host reference (relative to sum |a||w| of the output).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o split_lab split_lab.hip
#include "../csrc/gemm_x3.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  const char* name;
  int M, K, N, epi;
};

int main(int argc, char** argv) {
  const Shape shapes[] = {
      {"qkp d384", 49442, 384, 768, EPI_NONE},
      {"ffn_in d384", 49442, 384, 1280, EPI_SWOOSHL},
      {"ffn_out d384", 49442, 1280, 384, EPI_RESADD},
      {"ffn_in d256", 98813, 256, 960, EPI_SWOOSHL},
      {"ffn_out d256", 98813, 960, 256, EPI_RESADD},
      {"ffn_in d512", 24753, 512, 1920, EPI_SWOOSHL},
      {"embed out", 197561, 2432, 192, EPI_NONE},
      {"convnext pw1", 500000, 128, 384, EPI_SWOOSHL},
      {"convnext pw2", 500000, 384, 128, EPI_RESADD},
  };
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  uint32_t st = 12345u;
  auto nd = [&](std::mt19937&) {  // fast uniform in [-1.7, 1.7) (unit variance)
    st = st * 1664525u + 1013904223u;
    return ((st >> 8) * (1.0f / 16777216.0f) - 0.5f) * 3.4641f;
  };
  std::mt19937 rng(7);
  for (int si = 0; si < (int)(sizeof(shapes) / sizeof(shapes[0])); ++si) {
    if (only >= 0 && si != only) continue;
    const Shape& s = shapes[si];
    const size_t na = (size_t)s.M * s.K, nw = (size_t)s.N * s.K, nc = (size_t)s.M * s.N;
    std::vector<float> hA(na), hW(nw), hb(s.N), hC0(nc);
    for (auto& x : hA) x = nd(rng);
    const float ws = 1.f / std::sqrt((float)s.K);
    for (auto& x : hW) x = nd(rng) * ws;
    for (auto& x : hb) x = 0.1f * nd(rng);
    for (size_t i = 0; i < nc; i += 97) hC0[i] = nd(rng);
    float *dA, *dW, *db, *dC, *dC0;
    __bf16* dWx;
    hipMalloc(&dA, na * 4);
    hipMalloc(&dW, nw * 4);
    hipMalloc(&dWx, nw * 2 * 3);
    hipMalloc(&db, s.N * 4);
    hipMalloc(&dC, nc * 4);
    hipMalloc(&dC0, nc * 4);
    hipMemcpy(dA, hA.data(), na * 4, hipMemcpyHostToDevice);
    hipMemcpy(dW, hW.data(), nw * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, hb.data(), s.N * 4, hipMemcpyHostToDevice);
    hipMemcpy(dC0, hC0.data(), nc * 4, hipMemcpyHostToDevice);
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
    // f16x3 tile variants (all bit-identical: same 16-deep slabs in the same MFMA order
    // per output; BK = 32 changes nothing in the per-output order either)
    if (getenv("SPLIT_LAB_TILES")) {
      split_to_bf16(dW, dWx, (long)nw, kPiecesF16, 0);
      struct V {
        const char* name;
        void (*fn)(const GemmParams&, const __bf16*, long, hipStream_t);
      };
#define ZV(BM, BN, WM, WN, BK) \
  {#BM "x" #BN " w" #WM "x" #WN " bk" #BK, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) { \
     if (q.N % BN) return; \
     launch_x3_t<BM, BN, WM, WN, ALOAD_DENSE, EPI_NONE, 2, BK, 1>(q, b, lo, st); }}
#define ZG(NS, BN) \
  {"glds ns" #NS " bn" #BN, [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) { \
     if (q.N % BN || q.K % 32) return; \
     launch_glds_h3<NS, EPI_NONE, BN>(q, b, lo, st); }}
#define ZG4(NS, BN) \
  {"glds ns" #NS " bn" #BN " w4x1", [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) { \
     if (q.N % BN || q.K % 32) return; \
     launch_glds_h3<NS, EPI_NONE, BN, 4>(q, b, lo, st); }}
#define ZGR(NS, BN, WM) \
  {"glds ns" #NS " bn" #BN " wm" #WM " rb", [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) { \
     if (q.N % BN || q.K % 32) return; \
     launch_glds_h3<NS, EPI_NONE, BN, WM, 3, ALOAD_DENSE, 1>(q, b, lo, st); }}
      // "hi only": the glds loop with one MFMA per product instead of three (timing
      // diagnostic; its output differs by design)
      const V vars[] = {ZG(2, 128), ZV(128, 128, 2, 2, 32), ZGR(2, 128, 2), ZGR(3, 128, 2),
                        ZGR(2, 64, 4), ZGR(2, 128, 4), ZGR(3, 64, 2), ZG(2, 64), ZG4(2, 64),
                        {"glds ns2 bn128 hi only", [](const GemmParams& q, const __bf16* b, long lo, hipStream_t st) {
                           if (q.N % 128 || q.K % 32) return;
                           launch_glds_h3<2, EPI_NONE, 128, 2, 1>(q, b, lo, st); }}};
#undef ZG
#undef ZG4
#undef ZGR
#undef ZV
      std::vector<float> ref0;
      for (const V& v : vars) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipMemset(dC, 0, nc * 4);
        v.fn(p, dWx, (long)nw, 0);
        hipDeviceSynchronize();
        std::vector<float> got(nc);
        hipMemcpy(got.data(), dC, nc * 4, hipMemcpyDeviceToHost);
        if (ref0.empty()) ref0 = got;
        size_t ndiff = 0;
        for (size_t i = 0; i < nc; i += 7) ndiff += got[i] != ref0[i];
        for (int w = 0; w < 2; ++w) v.fn(p, dWx, (long)nw, 0);
        hipEventRecord(e0, 0);
        for (int it = 0; it < 10; ++it) v.fn(p, dWx, (long)nw, 0);
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 100.0;
        const double f32flops = 2.0 * s.M * s.K * s.N;
        printf("%-14s f16x3 %-20s %8.1f us  mfma %.3f of 2.5 PF  differs_from_first %zu\n", s.name,
               v.name, us, 3 * f32flops / us * 1e-6 / 2500.0, ndiff);
        fflush(stdout);
      }
      hipFree(dA); hipFree(dW); hipFree(dWx); hipFree(db); hipFree(dC); hipFree(dC0);
      continue;
    }
    for (int pieces : {3, kPiecesF16}) {
      split_to_bf16(dW, dWx, (long)nw, pieces, 0);
      auto run = [&]() {
        if (s.epi == EPI_RESADD) hipMemcpyAsync(dC, dC0, nc * 4, hipMemcpyDeviceToDevice, 0);
        gemm_x3(p, dWx, (long)nw, s.epi, ALOAD_DENSE, 0, pieces);
      };
      run();
      hipDeviceSynchronize();
      std::vector<float> hC(nc);
      hipMemcpy(hC.data(), dC, nc * 4, hipMemcpyDeviceToHost);
      double emax = 0.0;
      std::mt19937 r2(11);
      for (int t = 0; t < 512; ++t) {
        const long m = r2() % s.M, n = r2() % s.N;
        double acc = hb[n], mag = std::fabs(hb[n]);
        for (int k = 0; k < s.K; ++k) {
          acc += (double)hA[m * s.K + k] * hW[n * s.K + k];
          mag += std::fabs((double)hA[m * s.K + k] * hW[n * s.K + k]);
        }
        double ref = acc;
        if (s.epi == EPI_SWOOSHL) ref = std::log1p(std::exp(acc - 4.0)) - 0.08 * acc - 0.035;
        if (s.epi == EPI_RESADD) ref = acc + hC0[m * s.N + n];
        emax = std::max(emax, std::fabs(hC[m * s.N + n] - ref) / (mag + 1e-30));
      }
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int w = 0; w < 2; ++w) gemm_x3(p, dWx, (long)nw, s.epi, ALOAD_DENSE, 0, pieces);
      hipEventRecord(e0, 0);
      for (int it = 0; it < 10; ++it) gemm_x3(p, dWx, (long)nw, s.epi, ALOAD_DENSE, 0, pieces);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double us = ms * 100.0;
      const double f32flops = 2.0 * s.M * s.K * s.N;
      const int prods = pieces == 3 ? 6 : 3;
      printf("%-14s %-6s %8.1f us  f32-equiv %6.1f TF/s  mfma %7.1f TF/s (%.3f of 2.5 PF)  err %.2e\n",
             s.name, pieces == 3 ? "bf16x6" : "f16x3", us, f32flops / us * 1e-6,
             prods * f32flops / us * 1e-6, prods * f32flops / us * 1e-6 / 2500.0, emax);
      fflush(stdout);
    }
    hipFree(dA);
    hipFree(dW);
    hipFree(dWx);
    hipFree(db);
    hipFree(dC);
    hipFree(dC0);
  }
  return 0;
}
