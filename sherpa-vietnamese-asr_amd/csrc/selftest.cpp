// Kernel-level self-tests on host data (include/zasr.h zasr_selftest_*): the f16x3
// one-accumulator kernels and the bf16 fused FFN run alone on caller-supplied operands, so the tests can sweep the
// shapes and row counts the decode only reaches incidentally (tail tiles, M < 16, every K / D
// and epilogue) against a float64 product on the host.  Device 0 of the process, its null
// stream, synchronous; nothing here is on the decode path.
#include <cstring>
#include <memory>
#include <vector>

#include "common.h"
#include "gemm.h"
#include "kernels.h"

namespace zasr {
namespace {
struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t bytes) { ZASR_HIP_CHECK(hipMalloc(&p, bytes > 0 ? bytes : 4)); }
  ~DevBuf() { (void)hipFree(p); }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};
void up(DevBuf& d, const void* h, size_t bytes) {
  if (bytes) ZASR_HIP_CHECK(hipMemcpy(d.p, h, bytes, hipMemcpyHostToDevice));
}
}  // namespace

void selftest_gemm_h3r(int M, int K, int N, int epi, const float* A, const float* W,
                       const float* bias, float* C) {
  ZASR_REQUIRE(M >= 1, "selftest gemm_h3r: M >= 1");
  ZASR_REQUIRE(gemm_h3r_supported(K, N, epi), "selftest gemm_h3r: unsupported K / N / epilogue");
  ZASR_REQUIRE(ffn_h3_weights_ok(W, (long)N * K), "selftest gemm_h3r: |w| must stay below 31");
  const int ncol = epi == EPI_GLU ? N / 2 : N;
  std::vector<__bf16> pk(2 * (size_t)N * K);
  ffn_pack_h3_host(W, N, K, pk.data());
  DevBuf dA((size_t)M * K * 4), dW(pk.size() * 2), dB((size_t)N * 4), dC((size_t)M * ncol * 4);
  up(dA, A, (size_t)M * K * 4);
  up(dW, pk.data(), pk.size() * 2);
  if (bias) up(dB, bias, (size_t)N * 4);
  up(dC, C, (size_t)M * ncol * 4);  // the RESADD operand (and what rows past M would keep)
  gemm_h3r(dA.as<float>(), dW.p, bias ? dB.as<float>() : nullptr, dC.as<float>(), ncol, M, N, K,
           epi, nullptr);
  ZASR_HIP_CHECK(hipDeviceSynchronize());
  ZASR_HIP_CHECK(hipMemcpy(C, dC.p, (size_t)M * ncol * 4, hipMemcpyDeviceToHost));
}

void selftest_ffn_h3(int R, int D, int F, const float* Y, const float* W1, const float* b1,
                     const float* W2, const float* b2, const float* byp_orig,
                     const float* byp_scale, float* X) {
  ZASR_REQUIRE(R >= 1, "selftest ffn_h3: R >= 1");
  ZASR_REQUIRE(ffn_h3_supported(D, F), "selftest ffn_h3: unsupported model / feed-forward dim");
  ZASR_REQUIRE(ffn_h3_weights_ok(W1, (long)F * D) && ffn_h3_weights_ok(W2, (long)F * D),
               "selftest ffn_h3: |w| must stay below 31");
  std::vector<__bf16> p1(2 * (size_t)F * D), p2(p1.size());
  ffn_pack_h3_host(W1, F, D, p1.data());
  ffn_pack_h3_host(W2, D, F, p2.data());
  const size_t xb = (size_t)R * D * 4;
  DevBuf dY(xb), dX(xb), d1(p1.size() * 2), d2(p2.size() * 2), db1((size_t)F * 4),
      db2((size_t)D * 4), dbo(byp_orig ? xb : 4), dbs((size_t)D * 4);
  up(dY, Y, xb);
  up(dX, X, xb);
  up(d1, p1.data(), p1.size() * 2);
  up(d2, p2.data(), p2.size() * 2);
  up(db1, b1, (size_t)F * 4);
  up(db2, b2, (size_t)D * 4);
  if (byp_orig) {
    ZASR_REQUIRE(byp_scale != nullptr, "selftest ffn_h3: bypass needs its scale");
    up(dbo, byp_orig, xb);
    up(dbs, byp_scale, (size_t)D * 4);
  }
  launch_ffn_fused_h3(dX.as<float>(), R, D, F, d1.p, db1.as<float>(), d2.p, db2.as<float>(),
                      nullptr, byp_orig ? dbo.as<float>() : nullptr,
                      byp_orig ? dbs.as<float>() : nullptr, dY.as<float>());
  ZASR_HIP_CHECK(hipDeviceSynchronize());
  ZASR_HIP_CHECK(hipMemcpy(X, dX.p, xb, hipMemcpyDeviceToHost));
}

void selftest_ffn_bf16(int R, int D, int F, const float* W1, const float* b1, const float* W2,
                       const float* b2, const float* byp_orig, const float* byp_scale, float* X,
                       int form) {
  ZASR_REQUIRE(form == 0 || form == 1, "selftest ffn_bf16: form 0 (default route) or 1 (rows form)");
  ZASR_REQUIRE(R >= 1, "selftest ffn_bf16: R >= 1");
  ZASR_REQUIRE(ffn_fused_supported(D), "selftest ffn_bf16: unsupported model dim");
  // W1 [F][D] and W2 [D][F] in bf16; d >= 256 in MFMA-fragment order (the engine's wp)
  std::vector<__bf16> h1((size_t)F * D), h2((size_t)D * F);
  for (size_t i = 0; i < h1.size(); ++i) h1[i] = (__bf16)W1[i];
  for (size_t i = 0; i < h2.size(); ++i) h2[i] = (__bf16)W2[i];
  if (D >= 256) {
    std::vector<__bf16> p1(h1.size()), p2(h2.size());
    ffn_pack_host(h1.data(), F, D, p1.data());
    ffn_pack_host(h2.data(), D, F, p2.data());
    h1.swap(p1);
    h2.swap(p2);
  }
  const size_t xb = (size_t)R * D * 4;
  DevBuf dX(xb), d1(h1.size() * 2), d2(h2.size() * 2), db1((size_t)F * 4), db2((size_t)D * 4),
      dbo(byp_orig ? xb : 4), dbs((size_t)D * 4);
  up(dX, X, xb);
  up(d1, h1.data(), h1.size() * 2);
  up(d2, h2.data(), h2.size() * 2);
  up(db1, b1, (size_t)F * 4);
  up(db2, b2, (size_t)D * 4);
  if (byp_orig) {
    ZASR_REQUIRE(byp_scale != nullptr, "selftest ffn_bf16: bypass needs its scale");
    up(dbo, byp_orig, xb);
    up(dbs, byp_scale, (size_t)D * 4);
  }
  const int saved = ffn_rows_on();
  ffn_set_rows(form);
  try {
    launch_ffn_fused(dX.as<float>(), R, D, F, d1.p, db1.as<float>(), d2.p, db2.as<float>(), nullptr,
                     byp_orig ? dbo.as<float>() : nullptr, byp_orig ? dbs.as<float>() : nullptr);
  } catch (...) {
    ffn_set_rows(saved);
    throw;
  }
  ffn_set_rows(saved);
  ZASR_HIP_CHECK(hipDeviceSynchronize());
  ZASR_HIP_CHECK(hipMemcpy(X, dX.p, xb, hipMemcpyDeviceToHost));
}

}  // namespace zasr
