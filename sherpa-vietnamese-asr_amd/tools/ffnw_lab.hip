// ffn_wide_kernel check + timing (development tool): random X / W1 / W2, the kernel vs a host
// reference on sampled rows (bf16 X and H like the kernel, double accumulation), then the
// mean time of 20 launches on the bench's shapes.  make -C tools ffnw_lab && ./tools/ffnw_lab
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <vector>

#ifndef NO_STAMPS
#define ZASR_FFN_STAMPS 1
#endif
#include "../csrc/ffn_kernels.hip"

using namespace zasr;

static float bf(float x) { return (float)(__bf16)x; }
static double swl(double x) { double y = x - 4.0; return (y > 20 ? y : std::log1p(std::exp(y))) - 0.08 * x - 0.035; }

static void run(int D, int F, int R) {
  std::mt19937 g(D * 7919 + F);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> x((size_t)R * D), b1(F), b2(D);
  std::vector<__bf16> w1((size_t)F * D), w2((size_t)D * F);
  for (auto& v : x) v = nd(g);
  for (auto& v : b1) v = 0.1f * nd(g);
  for (auto& v : b2) v = 0.1f * nd(g);
  for (auto& v : w1) v = (__bf16)(nd(g) / std::sqrt((float)D));
  for (auto& v : w2) v = (__bf16)(nd(g) / std::sqrt((float)F));
  float *dX, *db1, *db2;
  __bf16 *dW1, *dW2;
  hipMalloc(&dX, x.size() * 4); hipMalloc(&db1, F * 4); hipMalloc(&db2, D * 4);
  hipMalloc(&dW1, w1.size() * 2); hipMalloc(&dW2, w2.size() * 2);
  hipMemcpy(dX, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db1, b1.data(), F * 4, hipMemcpyHostToDevice);
  hipMemcpy(db2, b2.data(), D * 4, hipMemcpyHostToDevice);
  {
    std::vector<__bf16> p1(w1.size()), p2(w2.size());
    ffn_pack_host(w1.data(), F, D, p1.data());
    ffn_pack_host(w2.data(), D, F, p2.data());
    hipMemcpy(dW1, p1.data(), w1.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW2, p2.data(), w2.size() * 2, hipMemcpyHostToDevice);
  }
  // both forms (ffn_rows_kernel / ffn_wide_kernel) from the same X: bit identity
  std::vector<float> y(x.size()), y0(x.size());
  for (int v = 0; v < 2; ++v) {
    g_ffnw_rows = 1 - v;
    hipMemcpy(dX, x.data(), x.size() * 4, hipMemcpyHostToDevice);
    launch_ffn_fused(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr);
    hipMemcpy(v == 0 ? y.data() : y0.data(), dX, y.size() * 4, hipMemcpyDeviceToHost);
  }
  const bool same = std::memcmp(y.data(), y0.data(), y.size() * 4) == 0;
  double err = 0, ref2 = 0;
  int rows = 0;
  for (int r = 0; r < R; r += (r < 130 ? 1 : 997)) {
    ++rows;
    std::vector<double> h(F);
    for (int j = 0; j < F; ++j) {
      double a = b1[j];
      for (int k = 0; k < D; ++k) a += (double)bf(x[(size_t)r * D + k]) * (float)w1[(size_t)j * D + k];
      h[j] = bf((float)swl(a));
    }
    for (int d = 0; d < D; ++d) {
      double o = b2[d];
      for (int j = 0; j < F; ++j) o += h[j] * (float)w2[(size_t)d * F + j];
      const double ref = x[(size_t)r * D + d] + o;
      err = std::fmax(err, std::fabs(ref - y[(size_t)r * D + d]));
      ref2 += o * o;
    }
  }
  const double rms = std::sqrt(ref2 / ((double)rows * D));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float best[2] = {1e30f, 1e30f};
  for (int rep = 0; rep < 3; ++rep)
    for (int v = 0; v < 2; ++v) {  // interleaved, best of 3: rows form, one block per tile
      g_ffnw_rows = 1 - v;
      for (int i = 0; i < 3; ++i) launch_ffn_fused(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr);
      hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) launch_ffn_fused(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best[v] = std::min(best[v], 1000.f * ms / 20);
    }
  g_ffnw_rows = 1;
  const float ms = best[0] * 20 / 1000.f;
  printf("  rows form %.1f us | one block per tile %.1f us  (%.3fx)  bit-identical %s\n", best[0], best[1],
         best[1] / best[0], same ? "yes" : "NO");
  const double us = 1000.0 * ms / 20, fl = 4.0 * R * D * F;
#ifdef ZASR_FFN_STAMPS
  {
    long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ffn_stamps), sizeof(st));
    printf("  stamps (shader cycles): stage %lld", st[1] - st[0]);
    for (int c = 0; c < 3; ++c)
      printf(" | c%d A %lld bar1 %lld write+bar2 %lld", c, st[3 + 4 * c] - st[2 + 4 * c], st[4 + 4 * c] - st[3 + 4 * c],
             st[5 + 4 * c] - st[4 + 4 * c]);
    printf(" | B0 %lld\n", st[6] - st[5]);
  }
#endif
  printf("D %d F %d R %d: max|err| %.3e (out rms %.3f, rows %d)  %.1f us  %.0f TFLOP/s (%.3f of 2.5 PF)  %.0f GB/s\n",
         D, F, R, err, rms, rows, us, fl / us / 1e6, fl / us / 1e6 / 2500.0, 12.0 * R * D / us / 1e3);
  hipFree(dX); hipFree(db1); hipFree(db2); hipFree(dW1); hipFree(dW2);
}

int main(int argc, char** argv) {
  run(384, 1280, 49442);
  run(384, 1024, 49442);
  run(384, 768, 49442);
  run(256, 960, 98813);
  run(256, 576, 98813);
  run(256, 768, 98813);
  run(512, 1920, 24753);
  run(512, 1536, 24753);
  run(512, 1152, 24753);
  run(384, 1280, 100);
  return 0;
}
