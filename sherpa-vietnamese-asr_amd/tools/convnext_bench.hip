// Development micro-benchmark (not part of libzasr): phases of the fused ConvNeXt kernel.
#include "../csrc/convnext_kernels.hip"

#include <cstdio>
#include <vector>

using namespace zasr;

template <int PH>
static float run(int rows, const float* x, const int* off, const int* map, const float* dw,
                 const float* db, const __bf16* w1, const float* b1, const __bf16* w2,
                 const float* b2, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int nb = (rows + 4) / 5;
  hipLaunchKernelGGL(convnext_fused_kernel<PH>, dim3(nb), dim3(256), 0, 0, x, off, map, rows, dw, db, w1, b1, w2, b2, out);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i)
    hipLaunchKernelGGL(convnext_fused_kernel<PH>, dim3(nb), dim3(256), 0, 0, x, off, map, rows, dw, db, w1, b1, w2, b2, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int rows = 197370;  // 50 Hz frames of 1 h of audio in 120 chunks
  const int nseq = 120;
  std::vector<int> off(nseq + 1), map(rows);
  for (int b = 0; b <= nseq; ++b) off[b] = (int)((long)rows * b / nseq);
  for (int b = 0; b < nseq; ++b)
    for (int r = off[b]; r < off[b + 1]; ++r) map[r] = b;
  float *x, *out, *dw, *db, *b1, *b2;
  __bf16 *w1, *w2;
  int *doff, *dmap;
  hipMalloc(&x, (size_t)rows * 19 * 128 * 4);
  hipMalloc(&out, (size_t)rows * 19 * 128 * 4);
  hipMalloc(&dw, 128 * 49 * 4);
  hipMalloc(&db, 128 * 4);
  hipMalloc(&b1, 384 * 4);
  hipMalloc(&b2, 128 * 4);
  hipMalloc(&w1, 384 * 128 * 2);
  hipMalloc(&w2, 128 * 384 * 2);
  hipMalloc(&doff, (nseq + 1) * 4);
  hipMalloc(&dmap, rows * 4);
  hipMemset(x, 0, (size_t)rows * 19 * 128 * 4);
  hipMemset(dw, 0, 128 * 49 * 4);
  hipMemset(db, 0, 128 * 4);
  hipMemset(b1, 0, 384 * 4);
  hipMemset(b2, 0, 128 * 4);
  hipMemset(w1, 0, 384 * 128 * 2);
  hipMemset(w2, 0, 128 * 384 * 2);
  hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dmap, map.data(), map.size() * 4, hipMemcpyHostToDevice);
  const double bytes = (double)rows * 19 * 128 * 4 * 2;
  float t1 = run<1>(rows, x, doff, dmap, dw, db, w1, b1, w2, b2, out);
  float t3 = run<3>(rows, x, doff, dmap, dw, db, w1, b1, w2, b2, out);
  float t5 = run<5>(rows, x, doff, dmap, dw, db, w1, b1, w2, b2, out);
  float t7 = run<7>(rows, x, doff, dmap, dw, db, w1, b1, w2, b2, out);
  printf("staging only        %8.3f ms\n", t1);
  printf("staging + dwconv    %8.3f ms\n", t3);
  printf("staging + MLP       %8.3f ms\n", t5);
  printf("all                 %8.3f ms  (%.0f GB/s of x in + out)\n", t7, bytes / t7 * 1e-6);
  return 0;
}
