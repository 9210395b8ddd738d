// Shared helpers for libzasr (host + device).  gfx950 / CDNA4 only.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#define ZASR_HIP_CHECK(expr)                                                          \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) {                                                           \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +    \
                               " at " + __FILE__ + ":" + std::to_string(__LINE__) +   \
                               " in " #expr);                                         \
    }                                                                                 \
  } while (0)

#define ZASR_REQUIRE(cond, msg)                                                       \
  do {                                                                                \
    if (!(cond)) throw std::runtime_error(std::string("zasr: ") + (msg));             \
  } while (0)

// Every kernel launch of the library goes through ZASR_LAUNCH: the launch, then the runtime's
// launch status (hipGetLastError: host-side, no synchronisation).  A refused launch (grid /
// block / LDS configuration, missing code object) throws, and the C ABI returns it as
// ZASR_ERR_RUNTIME with the HIP error in zasr_last_error() -- never a decode that goes on to
// read the stale workspace the kernel did not write.
#define ZASR_LAUNCH(...)                                                              \
  do {                                                                                \
    hipLaunchKernelGGL(__VA_ARGS__);                                                  \
    ::zasr::check_launch(__FILE__, __LINE__);                                         \
  } while (0)

namespace zasr {

// Grid of the persistent kernels (gemm_h3r, the fused f16x3 FFN: one block per CU, a per-CU
// share of the rows each).  While the pipelined decode runs other streams beside the encoder
// (the greedy pipeline's second encoder stream, the beam pipeline's J searches) they take 7/8
// of the CUs and leave the rest to those streams' kernels: f16x3 greedy 69.9k -> 70.7-70.9k
// xRT at 208-224 blocks of 256, config 3 in f16x3 58.5k -> 59.2k (profiles/r06/persist_ab/);
// a decode alone on the device keeps every CU.
// ZASR_PERSIST_CUS=N overrides (development A/B).
inline int& persist_share_flag() {
  static thread_local int on = 0;
  return on;
}
struct PersistShare {  // scoped: the calling thread's launches leave CUs to other streams
  int prev;
  explicit PersistShare(bool on) : prev(persist_share_flag()) { persist_share_flag() = on ? 1 : 0; }
  ~PersistShare() { persist_share_flag() = prev; }
  PersistShare(const PersistShare&) = delete;
  PersistShare& operator=(const PersistShare&) = delete;
};
inline int persist_blocks(int cus) {
  static const int cap = getenv("ZASR_PERSIST_CUS") != nullptr ? atoi(getenv("ZASR_PERSIST_CUS")) : -1;
  if (cap >= 0) return cap > 0 && cap < cus ? cap : cus;
  return persist_share_flag() ? cus - cus / 8 : cus;
}

inline void check_launch(const char* file, int line) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP kernel launch failed: ") + hipGetErrorString(e) +
                             " at " + file + ":" + std::to_string(line));
}

constexpr int kWave = 64;

__host__ __device__ inline int cdiv(int a, int b) { return (a + b - 1) / b; }
__host__ __device__ inline long cdivl(long a, long b) { return (a + b - 1) / b; }

// Activation functions (icefall scaling.py SwooshL/SwooshR ONNX forms).
__device__ __forceinline__ float softplusf(float x) {
  // log(1 + exp(x)), stable for large |x|
  return fmaxf(x, 0.f) + log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float swooshl(float x) { return softplusf(x - 4.f) - 0.08f * x - 0.035f; }
__device__ __forceinline__ float swooshr(float x) {
  return softplusf(x - 1.f) - 0.08f * x - 0.313261687f;
}
// native v_exp_f32 / v_log_f32 variants for the bf16-mode epilogues (abs error ~1e-7 vs the
// libm forms above).  The raw builtins skip the denormal range fix-ups __expf / __logf
// carry (v_cmp + 2 v_cndmask + v_ldexp per call): the log argument is in [1, 2] and an
// exp2 result that underflows only drops a term below 2^-126 -- 14 -> 9 VALU per element
// in the ConvNeXt / FFN / GEMM SwooshL epilogues, which are VALU-bound.
__device__ __forceinline__ float softplus_fast(float x) {
  constexpr float kLog2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  const float l = __builtin_amdgcn_logf(1.f + __builtin_amdgcn_exp2f(-fabsf(x) * kLog2e));
  return fmaf(l, kLn2, fmaxf(x, 0.f));
}
__device__ __forceinline__ float swooshl_fast(float x) {
  return softplus_fast(x - 4.f) - 0.08f * x - 0.035f;
}
__device__ __forceinline__ float swooshr_fast(float x) {
  return softplus_fast(x - 1.f) - 0.08f * x - 0.313261687f;
}
__device__ __forceinline__ float sigmoid_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-x * 1.4426950408889634f));
}
__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace zasr
