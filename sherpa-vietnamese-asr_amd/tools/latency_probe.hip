// Development probe (not part of libzasr): latency of the first global read of data written
// by the previous kernel launch, the pattern of the per-frame joiner -> search-step hand-off.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int S = 120, V = 2000;

__global__ void writer(float* out, int salt) {
  const int s = blockIdx.x;
  for (int v = threadIdx.x; v < V; v += 256) out[(long)s * V + v] = (float)(v ^ salt) * 1e-3f;
}

// thread 0 of each block stamps: start, after the row is loaded (8 float4 per lane)
__global__ void reader(const float* in, unsigned long long* stamps, float* sink, int mode) {
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  if (wid == 0) {
    const float4* r = reinterpret_cast<const float4*>(in + (long)s * V);
    float4 x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int i = lane + 64 * q;
      x[q] = i < V / 4 ? r[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) acc += x[q].x + x[q].y + x[q].z + x[q].w;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    stamps[s * 2] = t0;
    stamps[s * 2 + 1] = t1;
  }
  if (acc == 12345.f) sink[s] = acc;
}

__global__ void empty_kernel() {}

int main() {
  float *buf_a, *buf_b, *sink;
  unsigned long long* st;
  hipMalloc(&buf_a, (size_t)S * V * 4);
  hipMalloc(&buf_b, (size_t)S * V * 4);
  hipMalloc(&sink, S * 4);
  hipMalloc(&st, (size_t)S * 2 * 8);
  hipMemset(buf_a, 0, (size_t)S * V * 4);
  hipMemset(buf_b, 0, (size_t)S * V * 4);
  std::vector<unsigned long long> h(S * 2);
  auto report = [&](const char* name) {
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0, mx = 0;
    for (int s = 0; s < S; ++s) {
      double d = (double)(h[s * 2 + 1] - h[s * 2]);
      mean += d / S;
      if (d > mx) mx = d;
    }
    printf("%-44s load latency cycles: mean %8.0f  max %8.0f\n", name, mean, mx);
  };
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int it = 0; it < 3; ++it) {
    writer<<<S, 256>>>(buf_a, it);
    reader<<<S, 256>>>(buf_a, st, sink, 0);
    hipDeviceSynchronize();
    report("reader after writer (same buffer)");
    reader<<<S, 256>>>(buf_a, st, sink, 0);
    hipDeviceSynchronize();
    report("reader after reader (same buffer)");
    writer<<<S, 256>>>(buf_b, it);
    reader<<<S, 256>>>(buf_a, st, sink, 0);
    hipDeviceSynchronize();
    report("reader after writer (other buffer)");
    empty_kernel<<<1, 64>>>();
    reader<<<S, 256>>>(buf_a, st, sink, 0);
    hipDeviceSynchronize();
    report("reader after empty kernel");
  }
  // back-to-back pairs: wall time per (writer, reader) pair
  hipEventRecord(e0);
  for (int it = 0; it < 1000; ++it) {
    writer<<<S, 256>>>(buf_a, it);
    reader<<<S, 256>>>(buf_a, st, sink, 0);
  }
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("writer+reader pair: %.2f us\n", ms);
  report("last reader in the chain");
  hipEventRecord(e0);
  for (int it = 0; it < 1000; ++it) empty_kernel<<<S, 256>>>();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  printf("empty kernel (120 blocks) back to back: %.2f us each\n", ms);
  return 0;
}
