// Micro-benchmark of the split-bf16 GEMM (csrc/gemm_x3.hip) tile variants on the encoder's
// shapes (development tool, not part of libzasr).  Build: make -C tools x6_bench ; run on the
// GPU box: tools/x6_bench [pieces].  Per shape / variant: us per launch (median of 20 after 3
// warm-ups), TF/s of the split MFMA work (pieces' products x 2MKN), the fraction of the
// 2.5 PF bf16 peak, and the max relative error of 64 sampled outputs vs a host double
// reference of the f32 product.
#include "../csrc/gemm_x3.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  const char* name;
  int M, K, N, epi;
};

template <int NP>
struct Lab {
  float *dA, *dC, *dbias;
  __bf16* dB;
  std::vector<float> hA, hB, hbias;
  const Shape& s;
  Lab(const Shape& sh) : s(sh) {
    std::mt19937 rng(7);
    std::uniform_real_distribution<float> u(-1.f, 1.f);
    hA.resize((size_t)s.M * s.K);
    hB.resize((size_t)s.N * s.K);
    hbias.resize(s.N);
    for (auto& x : hA) x = u(rng);
    for (auto& x : hB) x = u(rng) / std::sqrt((float)s.K);
    for (auto& x : hbias) x = 0.1f * u(rng);
    hipMalloc(&dA, hA.size() * 4);
    hipMalloc(&dC, (size_t)s.M * s.N * 4);
    hipMalloc(&dbias, s.N * 4);
    float* dBf;
    hipMalloc(&dBf, hB.size() * 4);
    hipMalloc(&dB, hB.size() * 2 * NP);
    hipMemcpy(dA, hA.data(), hA.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dBf, hB.data(), hB.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dbias, hbias.data(), s.N * 4, hipMemcpyHostToDevice);
    split_to_bf16(dBf, dB, (long)hB.size(), NP, 0);
    hipDeviceSynchronize();
    hipFree(dBf);
  }
  ~Lab() {
    hipFree(dA);
    hipFree(dC);
    hipFree(dbias);
    hipFree(dB);
  }
  GemmParams params() const {
    GemmParams p{};
    p.A = dA;
    p.lda = s.K;
    p.sbk = 1;
    p.sbn = s.K;
    p.C = dC;
    p.ldc = s.N;
    p.bias = dbias;
    p.M = s.M;
    p.N = s.N;
    p.K = s.K;
    p.alpha = 1.f;
    p.max_M = s.M;
    return p;
  }
  template <typename F>
  void run(const char* tag, F launch) {
    const GemmParams p = params();
    hipMemset(dC, 0, (size_t)s.M * s.N * 4);
    launch(p, dB, (long)hB.size());
    hipDeviceSynchronize();
    std::mt19937 rng(5);
    double maxerr = 0;
    for (int q = 0; q < 64; ++q) {
      const int m = rng() % s.M, n = rng() % s.N;
      float g;
      hipMemcpy(&g, dC + (size_t)m * s.N + n, 4, hipMemcpyDeviceToHost);
      double ref = hbias[n], mag = std::fabs(hbias[n]);
      for (int k = 0; k < s.K; ++k) {
        const double t = (double)hA[(size_t)m * s.K + k] * hB[(size_t)n * s.K + k];
        ref += t;
        mag += std::fabs(t);
      }
      if (s.epi == EPI_SWOOSHL) ref = std::log1p(std::exp(ref - 4.0)) - 0.08 * ref - 0.035;
      maxerr = std::max(maxerr, std::fabs(g - ref) / std::max(1e-6, mag));
    }
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int w = 0; w < 3; ++w) launch(p, dB, (long)hB.size());
    std::vector<float> ts;
    for (int r = 0; r < 20; ++r) {
      hipEventRecord(a, 0);
      launch(p, dB, (long)hB.size());
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3;
    const double products = NP == 2 ? 3 : 6;
    const double tf = products * 2.0 * s.M * s.K * s.N / (us * 1e-6) / 1e12;
    printf("%-22s %-28s %9.1f us %7.1f TF/s %.3f of peak  err %.2e\n", s.name, tag, us, tf,
           tf / 2500.0, maxerr);
    fflush(stdout);
  }
};

#define VARIANT(BM, BN, WM, WN, BK)                                                          \
  lab.run(#BM "x" #BN " w" #WM "x" #WN " bk" #BK,                                            \
          [&](const GemmParams& p, const __bf16* B, long blo) {                               \
            if (sh.epi == EPI_SWOOSHL)                                                        \
              launch_x3_t<BM, BN, WM, WN, ALOAD_DENSE, EPI_SWOOSHL, NP, BK>(p, B, blo, 0);    \
            else if (sh.epi == EPI_RESADD)                                                    \
              launch_x3_t<BM, BN, WM, WN, ALOAD_DENSE, EPI_RESADD, NP, BK>(p, B, blo, 0);     \
            else                                                                              \
              launch_x3_t<BM, BN, WM, WN, ALOAD_DENSE, EPI_NONE, NP, BK>(p, B, blo, 0);       \
          })

template <int NP>
void sweep() {
  const Shape shapes[] = {
      {"ffn_in d384 F1280", 49442, 384, 1280, EPI_SWOOSHL},
      {"ffn_out d384 F1280", 49442, 1280, 384, EPI_RESADD},
      {"ffn_in d256 F960", 98813, 256, 960, EPI_SWOOSHL},
      {"proj d512 N1024", 24753, 512, 1024, EPI_NONE},
      {"qkp d384 N768", 49442, 384, 768, EPI_NONE},
      {"convnext pw1", 1000000, 128, 384, EPI_SWOOSHL},
      {"embed out K2432", 197561, 2432, 192, EPI_NONE},
  };
  printf("pieces %d\n", NP);
  for (const Shape& sh : shapes) {
    Lab<NP> lab(sh);
    VARIANT(128, 128, 2, 2, (NP == 2 ? 32 : 16));
    VARIANT(128, 128, 2, 2, 32);
    VARIANT(256, 128, 4, 2, 16);
    VARIANT(128, 256, 2, 4, 16);
    VARIANT(128, 128, 4, 2, 16);
  }
}

int main(int argc, char** argv) {
  const int pieces = argc > 1 ? atoi(argv[1]) : 3;
  if (pieces == 2)
    sweep<2>();
  else
    sweep<3>();
  return 0;
}
