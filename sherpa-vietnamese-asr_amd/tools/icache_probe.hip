// Development probe (not part of libzasr): cost of executing a large straight-line kernel body
// once per launch (instruction fetch) vs the same work in a small loop.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int S = 120;

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int N>
__global__ void bigcode(float* out, unsigned long long* st, float seed) {
  unsigned long long t0 = stamp();
  float a = seed + threadIdx.x, b = seed * 0.5f + blockIdx.x;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    a = fmaf(a, 1.0001f, b);
    b = fmaf(b, 0.9999f, a);
  }
  unsigned long long t1 = stamp();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 2] = t0;
    st[blockIdx.x * 2 + 1] = t1;
  }
  if (a == 12345.f) out[blockIdx.x] = a + b;
}

__global__ void smallcode(float* out, unsigned long long* st, float seed, int n) {
  unsigned long long t0 = stamp();
  float a = seed + threadIdx.x, b = seed * 0.5f + blockIdx.x;
  for (int i = 0; i < n; ++i) {
    a = fmaf(a, 1.0001f, b);
    b = fmaf(b, 0.9999f, a);
  }
  unsigned long long t1 = stamp();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 2] = t0;
    st[blockIdx.x * 2 + 1] = t1;
  }
  if (a == 12345.f) out[blockIdx.x] = a + b;
}

__global__ void other(float* out) { out[threadIdx.x] = threadIdx.x; }

int main() {
  float* out;
  unsigned long long* st;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&st, S * 2 * 8);
  std::vector<unsigned long long> h(S * 2);
  auto report = [&](const char* name) {
    hipDeviceSynchronize();
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int s = 0; s < S; ++s) mean += (double)(h[s * 2 + 1] - h[s * 2]) / S;
    printf("%-50s cycles %8.0f\n", name, mean);
  };
  for (int it = 0; it < 3; ++it) {
    bigcode<2048><<<S, 256>>>(out, st, 1.f);
    report("bigcode 4096 fma (cold)");
    bigcode<2048><<<S, 256>>>(out, st, 1.f);
    report("bigcode again (back to back)");
    other<<<1, 64>>>(out);
    bigcode<2048><<<S, 256>>>(out, st, 1.f);
    report("bigcode after another kernel");
    smallcode<<<S, 256>>>(out, st, 1.f, 2048);
    report("smallcode 4096 fma loop");
    other<<<1, 64>>>(out);
    smallcode<<<S, 256>>>(out, st, 1.f, 2048);
    report("smallcode after another kernel");
  }
  return 0;
}
