// ConvNeXt kernel timings (development tool): the bf16 MLP (convnext_mlp_kernel) and the
// depthwise 7x7 (convnext_dw_kernel, bf16 and f32), mean of 20 launches at the bench's sizes
// (1 h: 197,561 frames x 19 frequencies).  The round-6 A/Bs run with it (the MLP's staged
// epilogue, f32-staged and software-pipelined depthwise variants) are in
// profiles/r06/cnx_lab/.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o cnx_lab cnx_lab.hip
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../csrc/convnext_kernels.hip"

using namespace zasr;

static float run(long npos, const __bf16* y, const __bf16* x, const __bf16* w1, const float* b1,
                 const __bf16* w2, const float* b2, __bf16* out) {
  const dim3 grid((unsigned)cdivl(npos, 128));
  hipLaunchKernelGGL(convnext_mlp_kernel, grid, dim3(256), 0, 0, y, x, npos, w1, b1, w2, b2, out);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i)
    hipLaunchKernelGGL(convnext_mlp_kernel, grid, dim3(256), 0, 0, y, x, npos, w1, b1, w2, b2, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return 1000.f * ms / 20;
}

// depthwise 7x7, bf16 (64 channels per block) over 121 sequences
template <int C>
static float run_dw(int rows, const __bf16* x, const int* loff, const int* lmap, const float* w,
                    const float* b, __bf16* y) {
  const dim3 grid(cdiv(rows, kDwT), 128 / C);
  hipLaunchKernelGGL((convnext_dw_kernel<__bf16, C>), grid, dim3(256), 0, 0, x, loff, lmap, rows, w, b, y);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i)
    hipLaunchKernelGGL((convnext_dw_kernel<__bf16, C>), grid, dim3(256), 0, 0, x, loff, lmap, rows, w, b, y);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return 1000.f * ms / 20;
}

static float run_dw_f32(int rows, const float* x, const int* loff, const int* lmap, const float* w,
                        const float* b, float* y) {
  const dim3 grid(cdiv(rows, kDwT), 4);
  hipLaunchKernelGGL((convnext_dw_kernel<float, 32>), grid, dim3(256), 0, 0, x, loff, lmap, rows, w, b, y);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int i = 0; i < 20; ++i)
    hipLaunchKernelGGL((convnext_dw_kernel<float, 32>), grid, dim3(256), 0, 0, x, loff, lmap, rows, w, b, y);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return 1000.f * ms / 20;
}

static void dw_ab() {
  const int nseq = 121, rows = 197561;
  std::vector<int> loff(nseq + 1), lmap(rows);
  for (int b = 0; b <= nseq; ++b) loff[b] = (int)((long)rows * b / nseq);
  for (int b = 0; b < nseq; ++b)
    for (int r = loff[b]; r < loff[b + 1]; ++r) lmap[r] = b;
  std::mt19937 g(11);
  std::normal_distribution<float> nd(0.f, 1.f);
  const size_t n = (size_t)rows * 19 * 128;
  std::vector<__bf16> hx(n);
  for (auto& v : hx) v = (__bf16)nd(g);
  std::vector<float> w(128 * 49), b(128);
  for (auto& v : w) v = 0.15f * nd(g);
  for (auto& v : b) v = 0.1f * nd(g);
  __bf16 *dx, *y0, *y1, *y2;
  int *dlo, *dlm;
  float *dw, *db;
  hipMalloc(&dx, n * 2); hipMalloc(&y0, n * 2); hipMalloc(&y1, n * 2); hipMalloc(&y2, n * 2);
  hipMalloc(&dlo, loff.size() * 4); hipMalloc(&dlm, lmap.size() * 4);
  hipMalloc(&dw, w.size() * 4); hipMalloc(&db, b.size() * 4);
  hipMemcpy(dx, hx.data(), n * 2, hipMemcpyHostToDevice);
  hipMemcpy(dlo, loff.data(), loff.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dlm, lmap.data(), lmap.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, w.data(), w.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  const float t0 = run_dw<64>(rows, dx, dlo, dlm, dw, db, y0);
  printf("dw7x7 bf16 rows %d: %.1f us (%.0f GB/s)\n", rows, t0, 2.0 * n * 2 / t0 / 1e3);
  fflush(stdout);
  hipFree(y0); hipFree(y1); hipFree(y2);
  // f32 (the f16x3 / fp32 modes): 32 channels per block, 4 channel blocks
  {
    std::vector<float> hf(n);
    for (size_t i = 0; i < n; ++i) hf[i] = (float)hx[i] + 1e-3f * nd(g);
    float *fx, *f0, *f1;
    hipMalloc(&fx, n * 4); hipMalloc(&f0, n * 4); hipMalloc(&f1, n * 4);
    hipMemcpy(fx, hf.data(), n * 4, hipMemcpyHostToDevice);
    const float u0 = run_dw_f32(rows, fx, dlo, dlm, dw, db, f0);
    printf("dw7x7 f32 rows %d: %.1f us (%.0f GB/s)\n", rows, u0, 2.0 * n * 4 / u0 / 1e3);
    hipFree(fx); hipFree(f0); hipFree(f1);
  }
  hipFree(dx); hipFree(dlo); hipFree(dlm); hipFree(dw); hipFree(db);
}

int main() {
  dw_ab();
  for (long npos : {3753659L, 100003L, 127L}) {
    std::mt19937 g(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    std::vector<__bf16> hy(npos * 128), hx(npos * 128), w1(384 * 128), w2(128 * 384), p1(w1.size()),
        p2(w2.size());
    for (auto& v : hy) v = (__bf16)nd(g);
    for (auto& v : hx) v = (__bf16)nd(g);
    for (auto& v : w1) v = (__bf16)(nd(g) * 0.09f);
    for (auto& v : w2) v = (__bf16)(nd(g) * 0.05f);
    std::vector<float> b1(384), b2(128);
    for (auto& v : b1) v = 0.1f * nd(g);
    for (auto& v : b2) v = 0.1f * nd(g);
    pack_frag32_host(w1.data(), 384, 128, p1.data());
    pack_frag32_host(w2.data(), 128, 384, p2.data());
    __bf16 *dy, *dx, *dw1, *dw2, *o0, *o1;
    float *db1, *db2;
    const size_t nb = (size_t)npos * 128 * 2;
    hipMalloc(&dy, nb); hipMalloc(&dx, nb); hipMalloc(&o0, nb); hipMalloc(&o1, nb);
    hipMalloc(&dw1, p1.size() * 2); hipMalloc(&dw2, p2.size() * 2);
    hipMalloc(&db1, 384 * 4); hipMalloc(&db2, 128 * 4);
    hipMemcpy(dy, hy.data(), nb, hipMemcpyHostToDevice);
    hipMemcpy(dx, hx.data(), nb, hipMemcpyHostToDevice);
    hipMemcpy(dw1, p1.data(), p1.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dw2, p2.data(), p2.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(db1, b1.data(), 384 * 4, hipMemcpyHostToDevice);
    hipMemcpy(db2, b2.data(), 128 * 4, hipMemcpyHostToDevice);
    hipMemset(o0, 0, nb);
    hipMemset(o1, 0, nb);
    const float t0 = run(npos, dy, dx, dw1, db1, dw2, db2, o0);
    printf("convnext MLP npos %ld: %.1f us (%.0f GB/s of Y + x + out)\n", npos, t0, 3.0 * nb / t0 / 1e3);
    fflush(stdout);
    hipFree(dy); hipFree(dx); hipFree(o0); hipFree(o1); hipFree(dw1); hipFree(dw2);
    hipFree(db1); hipFree(db2);
  }
  return 0;
}
