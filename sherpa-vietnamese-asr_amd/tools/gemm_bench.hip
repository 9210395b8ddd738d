// Micro-benchmark of the bf16 projection GEMM on the encoder's shapes (development tool,
// not part of libzasr).  Build: make -C tools ; run on the GPU box: tools/gemm_bench
// Reports per shape/variant: us per launch, algorithmic GB/s (A + B + C [+ C read]) and TF/s,
// and the max relative error of 256 sampled outputs vs a host double reference.
#include "../csrc/gemm.hip"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  const char* name;
  int M, K, N, epi;
};

static float bf16r(float x) { return (float)(__bf16)x; }

template <int BK, typename TA, typename TC, int EPI>
static void run_variant(const char* tag, const Shape& s, float* dA, __bf16* dA16, __bf16* dB,
                        float* dC, __bf16* dC16, float* dbias, const std::vector<float>& hA,
                        const std::vector<float>& hB, const std::vector<float>& hbias) {
  GemmParams p{};
  p.A = std::is_same<TA, float>::value ? dA : reinterpret_cast<const float*>(dA16);
  p.lda = s.K;
  p.sbk = 1;
  p.sbn = s.K;
  p.C = std::is_same<TC, float>::value ? dC : reinterpret_cast<float*>(dC16);
  p.ldc = s.N;
  p.bias = dbias;
  p.M = s.M;
  p.N = s.N;
  p.K = s.K;
  p.alpha = 1.f;
  p.max_M = s.M;
  hipMemset(dC, 0, (size_t)s.M * s.N * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  launch_tile_h<BK, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0);
  hipDeviceSynchronize();
  // correctness (before timing, for RESADD C started at 0)
  std::vector<float> got(256);
  std::mt19937 rng(5);
  double maxerr = 0;
  for (int q = 0; q < 64; ++q) {
    int m = rng() % s.M, n = rng() % s.N;
    float g;
    if (std::is_same<TC, float>::value) {
      hipMemcpy(&g, dC + (size_t)m * s.N + n, 4, hipMemcpyDeviceToHost);
    } else {
      __bf16 h;
      hipMemcpy(&h, dC16 + (size_t)m * s.N + n, 2, hipMemcpyDeviceToHost);
      g = (float)h;
    }
    double ref = hbias[n];
    for (int k = 0; k < s.K; ++k) ref += (double)bf16r(hA[(size_t)m * s.K + k]) * bf16r(hB[(size_t)n * s.K + k]);
    if (EPI == EPI_SWOOSHL) ref = std::log1p(std::exp(ref - 4.0)) - 0.08 * ref - 0.035;
    double e = std::fabs(g - ref) / std::max(1.0, std::fabs(ref));
    maxerr = std::max(maxerr, e);
  }
  const int reps = 10;
  hipEventRecord(a, 0);
  for (int r = 0; r < reps; ++r) launch_tile_h<BK, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  double us = ms * 1000.0 / reps;
  double bytes = (double)s.M * s.K * sizeof(TA) + (double)s.N * s.K * 2 +
                 (double)s.M * s.N * sizeof(TC) * (EPI == EPI_RESADD ? 2 : 1);
  double flops = 2.0 * s.M * s.K * s.N;
  printf("%-8s %-22s M=%8d K=%5d N=%5d  %9.1f us  %7.0f GB/s  %6.1f TF/s  err %.2e\n", s.name,
         tag, s.M, s.K, s.N, us, bytes / us * 1e-3, flops / us * 1e-6, maxerr);
  hipEventDestroy(a);
  hipEventDestroy(b);
}

int main() {
  std::vector<Shape> shapes = {
      {"qkp384", 49442, 384, 768, EPI_NONE},   {"in864", 49442, 384, 864, EPI_NONE},
      {"in512", 98813, 256, 512, EPI_NONE},    {"in1024", 24753, 512, 1024, EPI_NONE},
      {"in192", 197561, 192, 384, EPI_NONE},   {"out1024", 49442, 1024, 384, EPI_RESADD},
      {"out384", 49442, 384, 384, EPI_RESADD}, {"out256", 98813, 256, 256, EPI_RESADD},
  };
  size_t maxA = 0, maxC = 0, maxB = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxB = std::max(maxB, (size_t)s.N * s.K);
  }
  float *dA, *dC, *dbias;
  __bf16 *dA16, *dB, *dC16;
  hipMalloc(&dA, maxA * 4);
  hipMalloc(&dA16, maxA * 2);
  hipMalloc(&dC, maxC * 4);
  hipMalloc(&dC16, maxC * 2);
  hipMalloc(&dB, maxB * 2);
  hipMalloc(&dbias, 4096 * 4);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> hA(maxA), hB(maxB), hbias(4096);
  for (auto& x : hA) x = nd(rng);
  for (auto& x : hB) x = nd(rng) * 0.08f;
  for (auto& x : hbias) x = nd(rng) * 0.1f;
  std::vector<__bf16> hA16(maxA), hB16(maxB);
  for (size_t i = 0; i < maxA; ++i) hA16[i] = (__bf16)hA[i];
  for (size_t i = 0; i < maxB; ++i) hB16[i] = (__bf16)hB[i];
  hipMemcpy(dA, hA.data(), maxA * 4, hipMemcpyHostToDevice);
  hipMemcpy(dA16, hA16.data(), maxA * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB16.data(), maxB * 2, hipMemcpyHostToDevice);
  hipMemcpy(dbias, hbias.data(), 4096 * 4, hipMemcpyHostToDevice);
  for (int deep = 0; deep < 2; ++deep) {
    gemm_set_deep(deep);
    for (auto& s : shapes) {
      if (s.epi == EPI_RESADD)
        run_variant<32, __bf16, float, EPI_RESADD>(deep ? "deep bf16A f32C" : "base bf16A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
      else {
        run_variant<32, float, __bf16, EPI_NONE>(deep ? "deep f32A bf16C" : "base f32A bf16C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        // the same projection from a bf16 copy of A (what a bf16 shadow of the residual
        // stream, written by its producer, would feed)
        if (deep)
          run_variant<32, __bf16, __bf16, EPI_NONE>("deep bf16A bf16C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
      }
    }
  }
  return 0;
}
