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
      {"pw1", 3750030, 128, 384, EPI_SWOOSHL}, {"pw2", 3750030, 384, 128, EPI_RESADD},
      {"ffin0", 197370, 192, 768, EPI_SWOOSHL}, {"ffout0", 197370, 768, 192, EPI_RESADD},
      {"ffout2", 49342, 1152, 384, EPI_RESADD}, {"inproj1", 98685, 256, 272, EPI_NONE},
      {"ffin3", 24671, 512, 1280, EPI_SWOOSHL},
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
  for (auto& s : shapes) {
    // A/B host copies must match the shape's (K) layout: reuse the prefix
    switch (s.epi) {
      case EPI_SWOOSHL:
        run_variant<32, float, float, EPI_SWOOSHL>("bk32 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, float, float, EPI_SWOOSHL>("bk64 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, float, __bf16, EPI_SWOOSHL>("bk64 f32A bf16C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        break;
      case EPI_RESADD:
        run_variant<32, float, float, EPI_RESADD>("bk32 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, float, float, EPI_RESADD>("bk64 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, __bf16, float, EPI_RESADD>("bk64 bf16A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        break;
      default:
        run_variant<32, float, float, EPI_NONE>("bk32 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, float, float, EPI_NONE>("bk64 f32A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        run_variant<64, __bf16, float, EPI_NONE>("bk64 bf16A f32C", s, dA, dA16, dB, dC, dC16, dbias, hA, hB, hbias);
        break;
    }
  }
  return 0;
}
