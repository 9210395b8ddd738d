// glu_dwconv1d_kernel timing (development tool): the ConvolutionModule depthwise conv over the
// bench hour's packed rows (121 sequences) at every stack's (rows, channels, kernel), f32 (the
// split modes: GLU already applied by the in_proj epilogue) and bf16, against the HBM roof of
// the bytes it must move (read rows x d, write rows x d).  make -C tools dw1_lab && ./tools/dw1_lab
#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <vector>

#include "../csrc/encoder_kernels.hip"

using namespace zasr;

static float time_launch(const std::function<void()>& f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0); hipEventDestroy(e1);
  return 1000.f * ms / 20;
}

static void run(int R, int d, int K) {
  std::mt19937 g(R + d + K);
  std::normal_distribution<float> nd(0.f, 1.f);
  const int S = 121;
  std::vector<int> off(S + 1), map(R);
  for (int b = 0; b <= S; ++b) off[b] = (int)((long)R * b / S);
  for (int b = 0; b < S; ++b)
    for (int r = off[b]; r < off[b + 1]; ++r) map[r] = b;
  std::vector<float> x((size_t)R * d), w((size_t)d * K), bias(d);
  for (auto& v : x) v = nd(g);
  for (auto& v : w) v = 0.2f * nd(g);
  for (auto& v : bias) v = 0.1f * nd(g);
  float *dx, *dy, *dw, *db;
  __bf16 *hx, *hy;
  int *doff, *dmap;
  hipMalloc(&dx, x.size() * 4); hipMalloc(&dy, x.size() * 4);
  hipMalloc(&hx, x.size() * 2); hipMalloc(&hy, x.size() * 2);
  hipMalloc(&dw, w.size() * 4); hipMalloc(&db, d * 4);
  hipMalloc(&doff, (S + 1) * 4); hipMalloc(&dmap, R * 4);
  hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  std::vector<__bf16> xh(x.size());
  for (size_t i = 0; i < x.size(); ++i) xh[i] = (__bf16)x[i];
  hipMemcpy(hx, xh.data(), xh.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, bias.data(), d * 4, hipMemcpyHostToDevice);
  hipMemcpy(doff, off.data(), (S + 1) * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmap, map.data(), R * 4, hipMemcpyHostToDevice);
  // check a few rows of the f32 path against the host
  launch_dwconv1d_post_glu(dx, doff, dmap, R, d, K, dw, db, dy, 0);
  hipDeviceSynchronize();
  std::vector<float> y(x.size());
  hipMemcpy(y.data(), dy, y.size() * 4, hipMemcpyDeviceToHost);
  double err = 0;
  for (int r = 0; r < R; r += 997) {
    const int b = map[r];
    for (int c = 0; c < d; ++c) {
      double a = bias[c];
      for (int k = 0; k < K; ++k) {
        const int t = r + k - K / 2;
        if (t >= off[b] && t < off[b + 1]) a += (double)w[(size_t)c * K + k] * x[(size_t)t * d + c];
      }
      const double sw = std::log1p(std::exp(a - 1.0)) - 0.08 * a - 0.313261687;
      err = std::fmax(err, std::fabs(sw - y[(size_t)r * d + c]));
    }
  }
  const float uf = time_launch([&] { launch_dwconv1d_post_glu(dx, doff, dmap, R, d, K, dw, db, dy, 0); });
  const float ub = time_launch([&] { launch_dwconv1d_post_glu_bf16(hx, doff, dmap, R, d, K, dw, db, hy, 0); });
  const double bf = 8.0 * R * d, bb = 4.0 * R * d;
  printf("R %6d d %3d K %2d: max|err| %.2e  f32 %6.1f us (%.2f of 8 TB/s)  bf16 %6.1f us (%.2f)\n", R, d, K,
         err, uf, bf / uf / 1e6 / 8000.0, ub, bb / ub / 1e6 / 8000.0);
  hipFree(dx); hipFree(dy); hipFree(hx); hipFree(hy); hipFree(dw); hipFree(db); hipFree(doff); hipFree(dmap);
}

int main() {
  run(197561, 192, 31);
  run(98813, 256, 31);
  run(49442, 384, 15);
  run(24753, 512, 15);
  return 0;
}
