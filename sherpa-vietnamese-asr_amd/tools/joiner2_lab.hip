// Joiner layout lab (development tool, not part of libzasr): logits[M][V] = J W^T + b for the
// speculative-greedy shapes (M = streams x window rows, V = 2000, D = 512, bf16).
//   base   = the production split-K kernel (search_kernels.hip joiner_bf16_kernel): 32 x 32
//            tiles, fragment-shaped loads of J and W straight from row-major buffers;
//   packed = J and W in MFMA-fragment order ([tile][k16][64 lanes][8 bf16], one coalesced
//            1 KB wave load per fragment); 128 x 64 block tile, W columns staged once in LDS
//            and shared by the 4 waves, each wave a 32-row tile with its whole K in registers.
// Each configuration is timed alone and behind a "pipeline" kernel that rewrites an 8 MB
// buffer (the search step between two joiner launches), minus that kernel alone.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <functional>
#include <random>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int D = 512, QK = D / 16;

__global__ __launch_bounds__(256) void base_kernel(const __bf16* J, const __bf16* W,
                                                   const float* bias, float* out, int M, int V) {
  constexpr int NK = 8;
  __shared__ float red[3 * 16 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32;
  const int n = blockIdx.x * 32 + col;
  const bool nv = n < V;
  const int ar = m0 + col < M ? m0 + col : M - 1;
  const int kb = wid * (D / 4) + 8 * h;
  const __bf16* arow = J + (long)ar * D + kb;
  const __bf16* brow = W + (long)(nv ? n : 0) * D + kb;
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
  if (wid > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wid - 1) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (wid != 0 || !nv) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] += red[r * 64 + lane] + red[(16 + r) * 64 + lane] + red[(32 + r) * 64 + lane];
  const float bb = bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < M) out[(long)row * V + n] = acc[r] + bb;
  }
}

// GC column groups of 32 per block (W staged in LDS), 4 waves = 4 row tiles of 32
template <int GC>
__global__ __launch_bounds__(256) void packed_kernel(const bf16x8* Jp, const bf16x8* Wp,
                                                     const float* bias, float* out, int M, int V) {
  __shared__ bf16x8 sW[GC * QK * 64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g0 = blockIdx.x * GC;
  const int rt = blockIdx.y * 4 + wid;
  const int m0 = rt * 32;
  const bool live = m0 < M;
  bf16x8 a[QK];
  if (live) {
#pragma unroll
    for (int q = 0; q < QK; ++q) a[q] = Jp[((long)rt * QK + q) * 64 + lane];
  }
  const bf16x8* src = Wp + (long)g0 * QK * 64;
#pragma unroll
  for (int i = 0; i < GC * QK * 64 / 256; ++i) sW[tid + 256 * i] = src[tid + 256 * i];
  __syncthreads();
  if (!live) return;
  f32x16 acc[GC];
#pragma unroll
  for (int j = 0; j < GC; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
#pragma unroll
  for (int q = 0; q < QK; ++q)
#pragma unroll
    for (int j = 0; j < GC; ++j)
      acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[q], sW[(j * QK + q) * 64 + lane], acc[j], 0, 0, 0);
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < GC; ++j) {
    const int col = (g0 + j) * 32 + (lane & 31);
    if (col >= V) continue;
    const float bb = bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (row < M) out[(long)row * V + col] = acc[j][r] + bb;
    }
  }
}

__global__ void pipeline_kernel(float* buf, long n, float salt) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    buf[i] = salt + (float)(i & 1023);
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

int main() {
  const int V = 2000, VG = 64;  // column groups padded to 64 (2048 columns)
  const int MMAX = 1920;
  std::mt19937 rng(3);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<__bf16> hJ((size_t)MMAX * D), hW((size_t)V * D);
  std::vector<float> hb(V);
  for (auto& x : hJ) x = (__bf16)std::tanh(nd(rng));
  for (auto& x : hW) x = (__bf16)(nd(rng) * 0.05f);
  for (auto& x : hb) x = nd(rng) * 0.1f;
  // packed images
  std::vector<__bf16> hJp((size_t)MMAX * D), hWp((size_t)VG * 32 * D, (__bf16)0.f);
  for (int row = 0; row < MMAX; ++row)
    for (int k = 0; k < D; ++k) {
      const int rt = row / 32, r = row % 32, q = k / 16, hh = (k % 16) / 8, j = k % 8;
      hJp[(((size_t)rt * QK + q) * 64 + r + 32 * hh) * 8 + j] = hJ[(size_t)row * D + k];
    }
  for (int n = 0; n < V; ++n)
    for (int k = 0; k < D; ++k) {
      const int g = n / 32, r = n % 32, q = k / 16, hh = (k % 16) / 8, j = k % 8;
      hWp[(((size_t)g * QK + q) * 64 + r + 32 * hh) * 8 + j] = hW[(size_t)n * D + k];
    }
  __bf16 *J, *W, *Jp, *Wp;
  float *bias, *out0, *out1, *buf;
  const long nbuf = 2L << 20;  // 8 MB
  hipMalloc(&J, hJ.size() * 2);
  hipMalloc(&W, hW.size() * 2);
  hipMalloc(&Jp, hJp.size() * 2);
  hipMalloc(&Wp, hWp.size() * 2);
  hipMalloc(&bias, V * 4);
  hipMalloc(&out0, (size_t)MMAX * V * 4);
  hipMalloc(&out1, (size_t)MMAX * V * 4);
  hipMalloc(&buf, nbuf * 4);
  hipMemcpy(J, hJ.data(), hJ.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(Jp, hJp.data(), hJp.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(Wp, hWp.data(), hWp.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(bias, hb.data(), V * 4, hipMemcpyHostToDevice);
  auto pipe = [&] { hipLaunchKernelGGL(pipeline_kernel, dim3(1024), dim3(256), 0, 0, buf, nbuf, 1.f); };
  const double t_pipe = time_it(pipe);
  printf("pipeline kernel alone %.2f us\n", t_pipe);
  for (int M : {120, 480, 960, 1920}) {
    auto base = [&] {
      hipLaunchKernelGGL(base_kernel, dim3((V + 31) / 32, (M + 31) / 32), dim3(256), 0, 0, J, W, bias, out0, M, V);
    };
    auto pk2 = [&] {
      hipLaunchKernelGGL(packed_kernel<2>, dim3(VG / 2, (M + 127) / 128), dim3(256), 0, 0,
                         reinterpret_cast<const bf16x8*>(Jp), reinterpret_cast<const bf16x8*>(Wp), bias, out1, M, V);
    };
    auto pk4 = [&] {
      hipLaunchKernelGGL(packed_kernel<4>, dim3(VG / 4, (M + 127) / 128), dim3(256), 0, 0,
                         reinterpret_cast<const bf16x8*>(Jp), reinterpret_cast<const bf16x8*>(Wp), bias, out1, M, V);
    };
    base();
    pk2();
    hipDeviceSynchronize();
    std::vector<float> o0((size_t)M * V), o1((size_t)M * V);
    hipMemcpy(o0.data(), out0, o0.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(o1.data(), out1, o1.size() * 4, hipMemcpyDeviceToHost);
    double err = 0;
    for (size_t i = 0; i < o0.size(); ++i) err = std::max(err, (double)std::fabs(o0[i] - o1[i]));
    const double tb = time_it(base), tp2 = time_it(pk2), tp4 = time_it(pk4);
    const double tbp = time_it([&] { pipe(); base(); }) - t_pipe;
    const double tp2p = time_it([&] { pipe(); pk2(); }) - t_pipe;
    const double tp4p = time_it([&] { pipe(); pk4(); }) - t_pipe;
    printf("M=%5d  alone: base %6.2f packed2 %6.2f packed4 %6.2f us | behind pipeline: base %6.2f packed2 %6.2f packed4 %6.2f us | max diff %.2e\n",
           M, tb, tp2, tp4, tbp, tp2p, tp4p, err);
  }
  return 0;
}
