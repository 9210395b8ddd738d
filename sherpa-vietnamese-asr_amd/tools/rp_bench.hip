// Multi-stage LDS-DMA GEMM (gemm.hip gemm_glds_kernel) vs the register-staged 128x128-tile
// bf16 GEMM on the
// Zipformer-68M projection shapes (development tool, not part of libzasr).
// Build: make -C tools rp_bench ; run on the GPU box: tools/rp_bench
// Per shape: us per launch and algorithmic GB/s of both kernels, and the max |diff| between
// their outputs relative to max(1, |ref|) (both bf16 operands, f32 accumulate).
#include "../csrc/gemm.hip"
#include "../csrc/gemm_rp.hip"

#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  const char* name;
  int M, K, N, epi;
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

static std::vector<float> fetch(const void* d, size_t n, bool bf16) {
  std::vector<float> out(n);
  if (bf16) {
    std::vector<__bf16> h(n);
    hipMemcpy(h.data(), d, n * 2, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < n; ++i) out[i] = (float)h[i];
  } else {
    hipMemcpy(out.data(), d, n * 4, hipMemcpyDeviceToHost);
  }
  return out;
}

int main() {
  std::vector<Shape> shapes = {
      {"attn_in0", 197370, 192, 272, EPI_NONE, false, true},
      {"na_in0", 197370, 192, 432, EPI_NONE, false, false},
      {"sa_in0", 197370, 192, 48, EPI_NONE, false, true},
      {"cv_in0", 197370, 192, 384, EPI_NONE, false, true},
      {"cv_out0", 197370, 192, 192, EPI_RESADD, true, false},
      {"na_out0", 197370, 144, 192, EPI_RESADD, true, false},
      {"sa_out0", 197370, 48, 192, EPI_RESADD, true, false},
      {"ff_in1", 98685, 256, 768, EPI_SWOOSHL, false, true},
      {"attn_in1", 98685, 256, 272, EPI_NONE, false, true},
      {"ff_in2", 49342, 384, 1024, EPI_SWOOSHL, false, true},
      {"cv_out2", 49342, 384, 384, EPI_RESADD, true, false},
      {"ff_in3", 24671, 512, 1536, EPI_SWOOSHL, false, true},
      {"na_out3", 24671, 384, 512, EPI_RESADD, true, false},
      {"enc_proj", 98685, 512, 512, EPI_NONE, false, false},
      {"ff_out1", 98685, 768, 256, EPI_RESADD, true, false},
      {"ff_out2", 49342, 1280, 384, EPI_RESADD, true, false},
      {"ff_out3", 24671, 1920, 512, EPI_RESADD, true, false},
      {"ff_in1b", 98685, 256, 960, EPI_SWOOSHL, false, true},
  };
  size_t maxA = 0, maxC = 0, maxB = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxB = std::max(maxB, (size_t)gemm_rp_packed_elems(s.N, s.K));
  }
  void *dA, *dA16, *dC0, *dC1, *dB, *dBp;
  float* dbias;
  hipMalloc(&dA, maxA * 4);
  hipMalloc(&dC0, maxC * 4);
  hipMalloc(&dC1, maxC * 4);
  hipMalloc(&dB, maxB * 2);
  hipMalloc(&dBp, maxB * 2);
  hipMalloc(&dbias, 4096 * 4);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  {
    std::vector<float> h(maxA);
    for (auto& x : h) x = nd(rng);
    hipMemcpy(dA, h.data(), maxA * 4, hipMemcpyHostToDevice);
    std::vector<__bf16> h16(maxA);
    for (size_t i = 0; i < maxA; ++i) h16[i] = (__bf16)h[i];
    hipMalloc(&dA16, maxA * 2);
    hipMemcpy(dA16, h16.data(), maxA * 2, hipMemcpyHostToDevice);
    std::vector<__bf16> hb(maxB);
    for (auto& x : hb) x = (__bf16)(nd(rng) * 0.06f);
    hipMemcpy(dB, hb.data(), maxB * 2, hipMemcpyHostToDevice);
    std::vector<float> hbias(4096);
    for (auto& x : hbias) x = nd(rng) * 0.1f;
    hipMemcpy(dbias, hbias.data(), 4096 * 4, hipMemcpyHostToDevice);
  }
  for (auto& s : shapes) {
    gemm_rp_pack_weights(dB, s.N, s.K, dBp, 0);
    GemmParams p{};
    p.A = reinterpret_cast<const float*>(s.a16 ? dA16 : dA);
    p.lda = s.K;
    p.sbk = 1;
    p.sbn = s.K;
    p.ldc = s.N;
    p.bias = dbias;
    p.M = s.M;
    p.N = s.N;
    p.K = s.K;
    p.alpha = 1.f;
    p.max_M = s.M;
    const size_t nC = (size_t)s.M * s.N;
    // same starting C for the residual epilogue
    hipMemset(dC0, 0, nC * 4);
    hipMemset(dC1, 0, nC * 4);
    p.C = reinterpret_cast<float*>(dC0);
    setenv("ZASR_GEMM_GLDS", "0", 1);
    gemm_bf16(p, dB, s.epi, ALOAD_DENSE, 0, s.a16, s.c16);
    setenv("ZASR_GEMM_GLDS", "2", 1);
    p.C = reinterpret_cast<float*>(dC1);
    gemm_bf16(p, dB, s.epi, ALOAD_DENSE, 0, s.a16, s.c16);
    hipDeviceSynchronize();
    auto r0 = fetch(dC0, nC, s.c16), r1 = fetch(dC1, nC, s.c16);
    double err = 0;
    for (size_t i = 0; i < nC; ++i)
      err = std::max(err, (double)std::fabs(r0[i] - r1[i]) / std::max(1.0, (double)std::fabs(r0[i])));
    setenv("ZASR_GEMM_GLDS", "0", 1);
    const double t_old = time_it([&] { gemm_bf16(p, dB, s.epi, ALOAD_DENSE, 0, s.a16, s.c16); });
    setenv("ZASR_GEMM_GLDS", "2", 1);
    const double t_rp = time_it([&] { gemm_bf16(p, dB, s.epi, ALOAD_DENSE, 0, s.a16, s.c16); });
    const double bytes = (double)s.M * s.K * (s.a16 ? 2 : 4) + (double)s.N * s.K * 2 +
                         (double)nC * (s.c16 ? 2 : 4) * (s.epi == EPI_RESADD ? 2 : 1);
    const double fl = 2.0 * s.M * s.K * s.N;
    printf("%-9s M=%7d K=%4d N=%5d %s%s  tile128 %7.1f us %5.0f GB/s | glds %7.1f us %5.0f GB/s %5.0f TF/s  x%.2f  diff %.2e\n",
           s.name, s.M, s.K, s.N, s.a16 ? "A16" : "A32", s.c16 ? "C16" : "C32", t_old,
           bytes / t_old * 1e-3, t_rp, bytes / t_rp * 1e-3, fl / t_rp * 1e-6, t_old / t_rp, err);
  }
  return 0;
}
