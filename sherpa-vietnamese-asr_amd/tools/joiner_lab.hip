// Joiner tile-shape lab (development tool, not part of libzasr): logits[M][V] = W J + b for
// the speculative-greedy shapes (M = streams x window rows, V = 2000, D = 512, bf16), with
// RT x CT output tiles of 32 x 32 per block and the K dimension split KW ways over waves.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int RT, int CT, int KW, int D, int DBG = 0>
__global__ __launch_bounds__(64 * RT * CT * KW) void jk(const __bf16* J, const __bf16* W,
                                                         const float* bias, float* out, int M,
                                                         int V) {
  constexpr int NK = D / KW / 16;  // k16 steps per wave
  __shared__ float red[(KW > 1 ? (KW - 1) : 1) * RT * CT * 16 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int kw = wid % KW, tile = wid / KW;
  const int rt = tile / CT, ct = tile % CT;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32 * RT + rt * 32;
  const int n = blockIdx.x * 32 * CT + ct * 32 + col;
  const bool nv = n < V;
  const int ar = m0 + col < M ? m0 + col : M - 1;
  const int kb = kw * (D / KW) + 8 * h;
  const __bf16* arow = J + (long)ar * D + kb;
  const __bf16* brow = ((DBG & 2) != 0 ? J + (long)ar * D : W + (long)(nv ? n : 0) * D) + kb;
  bf16x8 a[NK], b[NK];
#pragma unroll
  for (int q = 0; q < NK; ++q) {
    a[q] = *reinterpret_cast<const bf16x8*>(arow + 16 * q);
    b[q] = *reinterpret_cast<const bf16x8*>(brow + 16 * q);
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int q = 0; q < NK; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q], b[q], acc, 0, 0, 0);
  if constexpr (KW > 1) {
    if (kw > 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) red[(((kw - 1) * RT * CT + tile) * 16 + r) * 64 + lane] = acc[r];
    }
    __syncthreads();
    if (kw != 0) return;
#pragma unroll
    for (int w = 1; w < KW; ++w)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += red[(((w - 1) * RT * CT + tile) * 16 + r) * 64 + lane];
  }
  if (!nv) return;
  if constexpr ((DBG & 1) != 0) {
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) sum += acc[r];
    if (sum == 1234.5f) out[n] = sum;
    return;
  }
  const float bb = bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < M) out[(long)row * V + n] = acc[r] + bb;
  }
}

// each wave: RW row tiles sharing one set of W fragments (W read once per RW*32 rows)
template <int RW, int KW, int D>
__global__ __launch_bounds__(64 * KW) void jk2(const __bf16* J, const __bf16* W, const float* bias,
                                               float* out, int M, int V) {
  constexpr int NK = D / KW / 16;
  __shared__ float red[(KW > 1 ? (KW - 1) : 1) * RW * 16 * 64];
  const int lane = threadIdx.x & 63, kw = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32 * RW;
  const int n = blockIdx.x * 32 + col;
  const bool nv = n < V;
  const int kb = kw * (D / KW) + 8 * h;
  const __bf16* brow = W + (long)(nv ? n : 0) * D + kb;
  bf16x8 a[RW][NK], b[NK];
#pragma unroll
  for (int q = 0; q < NK; ++q) b[q] = *reinterpret_cast<const bf16x8*>(brow + 16 * q);
#pragma unroll
  for (int t = 0; t < RW; ++t) {
    const int ar = m0 + 32 * t + col < M ? m0 + 32 * t + col : M - 1;
#pragma unroll
    for (int q = 0; q < NK; ++q) a[t][q] = *reinterpret_cast<const bf16x8*>(J + (long)ar * D + kb + 16 * q);
  }
  f32x16 acc[RW];
#pragma unroll
  for (int t = 0; t < RW; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
    for (int q = 0; q < NK; ++q) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[t][q], b[q], acc[t], 0, 0, 0);
  }
  if constexpr (KW > 1) {
    if (kw > 0) {
#pragma unroll
      for (int t = 0; t < RW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(((kw - 1) * RW + t) * 16 + r) * 64 + lane] = acc[t][r];
    }
    __syncthreads();
    if (kw != 0) return;
#pragma unroll
    for (int w = 1; w < KW; ++w)
#pragma unroll
      for (int t = 0; t < RW; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] += red[(((w - 1) * RW + t) * 16 + r) * 64 + lane];
  }
  if (!nv) return;
  const float bb = bias[n];
#pragma unroll
  for (int t = 0; t < RW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < M) out[(long)row * V + n] = acc[t][r] + bb;
    }
}

static double time_it(const std::function<void()>& f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  hipEventRecord(a, 0);
  for (int r = 0; r < 200; ++r) f();
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.0 / 200;
}

template <int RW, int KW>
static double run2(const __bf16* J, const __bf16* W, const float* bias, float* out, int M, int V) {
  dim3 grid((V + 31) / 32, (M + 32 * RW - 1) / (32 * RW));
  return time_it([&] { hipLaunchKernelGGL((jk2<RW, KW, 512>), grid, dim3(64 * KW), 0, 0, J, W, bias, out, M, V); });
}

template <int RT, int CT, int KW, int DBG = 0>
static double run(const __bf16* J, const __bf16* W, const float* bias, float* out, int M, int V) {
  dim3 grid((V + 32 * CT - 1) / (32 * CT), (M + 32 * RT - 1) / (32 * RT));
  return time_it([&] { hipLaunchKernelGGL((jk<RT, CT, KW, 512, DBG>), grid, dim3(64 * RT * CT * KW), 0, 0, J, W, bias, out, M, V); });
}

int main() {
  const int V = 2000, D = 512;
  __bf16 *J, *W;
  float *bias, *out;
  hipMalloc(&J, 1024 * D * 2);
  hipMalloc(&W, V * D * 2);
  hipMalloc(&bias, V * 4);
  hipMalloc(&out, 1024L * V * 4);
  hipMemset(J, 0, 1024 * D * 2);
  hipMemset(W, 0, V * D * 2);
  hipMemset(bias, 0, V * 4);
  for (int M : {120, 240, 480, 960}) {
    printf("M=%4d  base %6.2f  rw2k4 %6.2f  rw4k4 %6.2f  rw2k8 %6.2f  rw4k8 %6.2f us\n", M,
           run<1, 1, 4, 0>(J, W, bias, out, M, V), run2<2, 4>(J, W, bias, out, M, V),
           run2<4, 4>(J, W, bias, out, M, V), run2<2, 8>(J, W, bias, out, M, V),
           run2<4, 8>(J, W, bias, out, M, V));
  }
  return 0;
}
