// ffn_wide_h3_kernel check + timing (development tool): random f32 X / W1 / W2, the f16x3 fused
// FFN vs a host double reference on sampled rows (exact f32 inputs: the error is the f16x3
// format's plus swooshl_fast's), then the mean time of 20 launches on the bench's shapes,
// beside the bf16 ffn_wide_kernel on the same shape.  make -C tools ffnh3_lab && ./tools/ffnh3_lab
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#ifndef NO_STAMPS
#define ZASR_FFN_STAMPS 1
#endif
#include "../csrc/ffn_kernels.hip"

using namespace zasr;

static double swl(double x) { double y = x - 4.0; return (y > 20 ? y : std::log1p(std::exp(y))) - 0.08 * x - 0.035; }

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

static void run(int D, int F, int R, bool sepY = false) {
  std::mt19937 g(D * 7919 + F);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> x((size_t)R * D), b1(F), b2(D), w1((size_t)F * D), w2((size_t)D * F);
  for (auto& v : x) v = nd(g);
  for (auto& v : b1) v = 0.1f * nd(g);
  for (auto& v : b2) v = 0.1f * nd(g);
  for (auto& v : w1) v = nd(g) / std::sqrt((float)D);
  for (auto& v : w2) v = nd(g) / std::sqrt((float)F);
  float *dX, *db1, *db2;
  __bf16 *dW1, *dW2, *dH1, *dH2;
  hipMalloc(&dX, x.size() * 4); hipMalloc(&db1, F * 4); hipMalloc(&db2, D * 4);
  hipMalloc(&dW1, w1.size() * 4); hipMalloc(&dW2, w2.size() * 4);
  hipMalloc(&dH1, w1.size() * 2); hipMalloc(&dH2, w2.size() * 2);
  hipMemcpy(dX, x.data(), x.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db1, b1.data(), F * 4, hipMemcpyHostToDevice);
  hipMemcpy(db2, b2.data(), D * 4, hipMemcpyHostToDevice);
  {
    std::vector<__bf16> p1(2 * w1.size()), p2(2 * w2.size());
    ffn_pack_h3_host(w1.data(), F, D, p1.data());
    ffn_pack_h3_host(w2.data(), D, F, p2.data());
    hipMemcpy(dW1, p1.data(), p1.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dW2, p2.data(), p2.size() * 2, hipMemcpyHostToDevice);
    std::vector<__bf16> h1(w1.size()), h2(w2.size()), q1(w1.size()), q2(w2.size());
    for (size_t i = 0; i < w1.size(); ++i) h1[i] = (__bf16)w1[i];
    for (size_t i = 0; i < w2.size(); ++i) h2[i] = (__bf16)w2[i];
    ffn_pack_host(h1.data(), F, D, q1.data());
    ffn_pack_host(h2.data(), D, F, q2.data());
    hipMemcpy(dH1, q1.data(), q1.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dH2, q2.data(), q2.size() * 2, hipMemcpyHostToDevice);
  }
  // sepY: the rows read (Y) are a second buffer, X only the residual (the ConvNeXt MLP form)
  float* dY = nullptr;
  std::vector<float> yv;
  if (sepY) {
    yv.resize(x.size());
    for (auto& v : yv) v = nd(g);
    hipMalloc(&dY, yv.size() * 4);
    hipMemcpy(dY, yv.data(), yv.size() * 4, hipMemcpyHostToDevice);
  }
  launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr, dY);
  hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) { printf("launch failed: %s\n", hipGetErrorString(e)); exit(1); }
  std::vector<float> y(x.size());
  hipMemcpy(y.data(), dX, y.size() * 4, hipMemcpyDeviceToHost);
  double err = 0, ref2 = 0;
  int rows = 0;
  // every row when the shape is small (the last block's tail included), else a sample
  const bool all_rows = (double)R * D * F < 4e9;
  long worst = -1;
  for (int r = 0; r < R; r += (all_rows || r < 130 || r >= R - 130 ? 1 : 997)) {
    ++rows;
    std::vector<double> h(F);
    for (int j = 0; j < F; ++j) {
      double a = b1[j];
      const float* in = sepY ? yv.data() : x.data();
      for (int k = 0; k < D; ++k) a += (double)in[(size_t)r * D + k] * w1[(size_t)j * D + k];
      h[j] = swl(a);
    }
    for (int d = 0; d < D; ++d) {
      double o = b2[d];
      for (int j = 0; j < F; ++j) o += h[j] * w2[(size_t)d * F + j];
      const double ref = x[(size_t)r * D + d] + o;
      if (std::fabs(ref - y[(size_t)r * D + d]) > err) worst = r;
      err = std::fmax(err, std::fabs(ref - y[(size_t)r * D + d]));
      ref2 += o * o;
    }
  }
  // last row (tail tile) too
  const double rms = std::sqrt(ref2 / ((double)rows * D));
  const float ub = time_launch([&] { launch_ffn_fused(dX, R, D, F, dH1, db1, dH2, db2, 0, nullptr, nullptr); });
  // split barriers (default) against block barriers: bit-identical outputs, interleaved
  // timings (the clock state drifts between back-to-back timings), best of 3 each
  bool same_sb = true;
  {
    float* dX2;
    hipMalloc(&dX2, x.size() * 4);
    hipMemcpy(dX2, x.data(), x.size() * 4, hipMemcpyHostToDevice);
    ffn_h3_set_split(0);
    launch_ffn_fused_h3(dX2, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr, dY);
    ffn_h3_set_split(1);
    std::vector<float> y0(x.size());
    hipMemcpy(y0.data(), dX2, y0.size() * 4, hipMemcpyDeviceToHost);
    same_sb = memcmp(y0.data(), y.data(), y.size() * 4) == 0;
    hipFree(dX2);
  }
  float us_bar = 1e30f, us = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    ffn_h3_set_split(0);
    us_bar = std::min(us_bar, time_launch([&] { launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr); }));
    ffn_h3_set_split(1);
    us = std::min(us, time_launch([&] { launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr); }));
  }
  printf("  block barriers %.1f us -> split barriers %.1f us (%s)\n", us_bar, us,
         same_sb ? "bit-identical" : "OUTPUTS DIFFER");
  const double fl = 4.0 * R * D * F;
#ifdef ZASR_FFN_STAMPS
  {
    long long st[80];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_ffn_stamps), sizeof(st));
    printf("  block 0 (shader cycles): X tile %lld", st[1] - st[0]);
    for (int c = 0; c < (F + 127) / 128 && c < 12; ++c)
      printf(" | c%d A %lld swl %lld B %lld", c, st[9 + 4 * c] - st[8 + 4 * c], st[10 + 4 * c] - st[9 + 4 * c],
             st[11 + 4 * c] - st[10 + 4 * c]);
    printf("\n");
    // per tile of block 0: X staging, chunk phases summed, epilogue (shader cycles)
    static long long ts[4896];
    hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_ffn_stamps), sizeof(ts));
    const int nch = (F + 127) / 128;
    for (int k = 0; k < 30; ++k) {
      const long long* t = ts + 1000 + 100 * k;
      if (t[0] == 0 || t[90] == 0 || t[90] < t[0]) break;
      long long a = 0, w = 0, b = 0;
      for (int c = 0; c < nch && c < 16; ++c) {
        a += t[3 + 4 * c] - t[2 + 4 * c];
        w += t[4 + 4 * c] - t[3 + 4 * c];
        b += t[5 + 4 * c] - t[4 + 4 * c];
      }
      const long long last = t[5 + 4 * ((nch - 1) & 15)];
      printf("    tile %d: total %lld | X %lld | A %lld swl %lld B %lld | epilogue %lld | gap to next %lld\n", k,
             t[90] - t[0], t[1] - t[0], a, w, b, t[90] - last,
             (k + 1 < 30 && ts[1000 + 100 * (k + 1)] > t[90]) ? ts[1000 + 100 * (k + 1)] - t[90] : -1);
    }
    // every wave of block 0, tile 1: A start / A end / H barrier passed / B end, per chunk,
    // relative to the earliest A start of the chunk
    for (int c = 0; c < nch && c < 4; ++c) {
      long long t0w = 1LL << 62;
      for (int w = 0; w < 8; ++w) t0w = std::min(t0w, ts[4000 + 100 * w + 4 * c]);
      printf("    tile 1 chunk %d per wave (A start, A end, H ready, B end):", c);
      for (int w = 0; w < 8; ++w) {
        const long long* q = ts + 4000 + 100 * w + 4 * c;
        printf(" w%d %lld/%lld/%lld/%lld", w, q[0] - t0w, q[1] - t0w, q[2] - t0w, q[3] - t0w);
      }
      printf("\n");
    }
    memset(ts, 0, sizeof(ts));
    hipMemcpyToSymbol(HIP_SYMBOL(g_ffn_stamps), ts, sizeof(ts));
  }
#endif
  if (dY) hipFree(dY);
  printf("  worst row %ld of %d\n", worst, R);
  printf("%sD %d F %d R %d: max|err| %.3e (out rms %.3f, rel %.2e, rows %d)  h3 %.1f us = %.3f of the fp16 peak "
         "(3 MFMA / product)  | bf16 %.1f us (%.3f)  ratio %.2f\n",
         sepY ? "(Y) " : "", D, F, R, err, rms, err / rms, rows, us, 3 * fl / us / 1e6 / 2500.0, ub, fl / ub / 1e6 / 2500.0, us / ub);
  fflush(stdout);
  hipFree(dX); hipFree(db1); hipFree(db2); hipFree(dW1); hipFree(dW2); hipFree(dH1); hipFree(dH2);
}

// the ConvNeXt MLP (d = 128, F = 384, Y separate) at other tile heights / split barriers /
// batched epilogue, against the engine's instance: bit-identical outputs, interleaved timings
template <int TU, bool SB, bool EB>
static float cnx_variant(float* X, int R, const __bf16* w1, const float* b1, const __bf16* w2,
                         const float* b2, const float* Y, bool time_it) {
  const int rpb = 16 * cdiv(cdiv(R, 256), 16);
  const dim3 grid(cdiv(R, rpb));
  auto go = [&] {
    hipLaunchKernelGGL((ffn_wide_h3_kernel<128, TU, 1, 8, SB, EB>), grid, dim3(512), 0, 0, X, R, 384, w1,
                       b1, w2, b2, nullptr, nullptr, rpb, Y);
  };
  if (!time_it) { go(); hipDeviceSynchronize(); return 0.f; }
  return time_launch(go);
}

static void cnx_mode() {
  const int D = 128, F = 384, R = 3753659;
  std::mt19937 g(5);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> x((size_t)R * D), y((size_t)R * D), b1(F), b2(D), w1((size_t)F * D), w2((size_t)D * F);
  for (auto& v : x) v = nd(g);
  for (auto& v : y) v = nd(g);
  for (auto& v : b1) v = 0.1f * nd(g);
  for (auto& v : b2) v = 0.1f * nd(g);
  for (auto& v : w1) v = nd(g) / std::sqrt((float)D);
  for (auto& v : w2) v = nd(g) / std::sqrt((float)F);
  std::vector<__bf16> p1(2 * w1.size()), p2(2 * w2.size());
  ffn_pack_h3_host(w1.data(), F, D, p1.data());
  ffn_pack_h3_host(w2.data(), D, F, p2.data());
  float *dX, *dY, *db1, *db2;
  __bf16 *dW1, *dW2;
  hipMalloc(&dX, x.size() * 4); hipMalloc(&dY, y.size() * 4); hipMalloc(&db1, F * 4); hipMalloc(&db2, D * 4);
  hipMalloc(&dW1, p1.size() * 2); hipMalloc(&dW2, p2.size() * 2);
  hipMemcpy(dY, y.data(), y.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(db1, b1.data(), F * 4, hipMemcpyHostToDevice);
  hipMemcpy(db2, b2.data(), D * 4, hipMemcpyHostToDevice);
  hipMemcpy(dW1, p1.data(), p1.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dW2, p2.data(), p2.size() * 2, hipMemcpyHostToDevice);
  std::vector<float> ref(x.size()), got(x.size());
  auto fresh = [&] { hipMemcpy(dX, x.data(), x.size() * 4, hipMemcpyHostToDevice); };
  fresh();
  launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr, dY);
  hipMemcpy(ref.data(), dX, ref.size() * 4, hipMemcpyDeviceToHost);
  struct V { const char* name; std::function<float(bool)> f; float best; };
  std::vector<V> vs = {
      {"engine (TU 8, block barriers)", [&](bool t) { return t ? time_launch([&] { launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr, dY); }) : (launch_ffn_fused_h3(dX, R, D, F, dW1, db1, dW2, db2, 0, nullptr, nullptr, dY), 0.f); }, 1e30f},
      {"TU 8 SB", [&](bool t) { return cnx_variant<8, true, false>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 8 EB", [&](bool t) { return cnx_variant<8, false, true>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 7", [&](bool t) { return cnx_variant<7, false, false>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 7 SB", [&](bool t) { return cnx_variant<7, true, false>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 6 SB", [&](bool t) { return cnx_variant<6, true, false>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 6 SB EB", [&](bool t) { return cnx_variant<6, true, true>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
      {"TU 5 SB EB", [&](bool t) { return cnx_variant<5, true, true>(dX, R, dW1, db1, dW2, db2, dY, t); }, 1e30f},
  };
  for (auto& v : vs) {
    fresh();
    v.f(false);
    hipMemcpy(got.data(), dX, got.size() * 4, hipMemcpyDeviceToHost);
    printf("  %-32s %s\n", v.name, memcmp(got.data(), ref.data(), got.size() * 4) ? "OUTPUTS DIFFER" : "bit-identical");
  }
  for (int rep = 0; rep < 3; ++rep)
    for (auto& v : vs) v.best = std::min(v.best, v.f(true));
  for (auto& v : vs) printf("  %-32s %.1f us\n", v.name, v.best);
  fflush(stdout);
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "cnx")) {
    cnx_mode();
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "sb")) {  // the bench's shapes
    run(384, 1024, 49442);
    run(384, 1280, 49442);
    run(384, 768, 49442);
    run(256, 768, 98813);
    run(256, 960, 98813);
    run(256, 576, 98813);
    run(192, 512, 197614);
    run(128, 384, 3753659, true);
    run(512, 1536, 24753);  // control: two H buffers, block barriers in both arms
    run(384, 1280, 3029);   // small shapes: tails, one tile
    run(128, 384, 100, true);
    run(192, 512, 100);
    return 0;
  }
  if (argc > 1 && !strcmp(argv[1], "tiles")) {  // the bench's largest shapes, per-tile stamps
    run(384, 1024, 49442);
    run(256, 768, 98813);
    run(512, 1536, 24753);
    run(128, 384, 3753659, true);
    return 0;
  }
  run(128, 384, 100, true);
  run(128, 384, 100);
  // the last block's remainder a whole TUM-group tile (rows past R clamped): rpb 224, 60 left
  run(128, 384, 57180, true);
  run(384, 1280, 57180);
  run(512, 1536, 24680);        // rpb 112 on 48-row tiles, 40 left
  run(192, 512, 39960);         // rpb 80 on 48-row tiles (two blocks per CU), 40 left
  run(128, 384, 7068, true);    // rpb 32: every block one 32-row tile
  run(128, 384, 11000, true);   // rpb 48: one 48-row tile
  run(384, 1280, 7068);
  run(256, 768, 7068);
  run(128, 384, 57503, true);   // an M-set-like row count (not a multiple of 16)
  run(128, 384, 57503);
  run(384, 1280, 3029);
  run(128, 384, 45056, true);   // rpb 176: two 64-row tiles + a 48-row tail
  run(128, 384, 36864, true);   // rpb 144: two 64-row tiles + a 16-row tail
  run(128, 384, 28672, true);   // rpb 112: one 64-row tile + a 48-row tail
  run(384, 1280, 45056);        // rpb 176: 48-row tail
  run(384, 1280, 20480);        // rpb 80: 64 + 16
  run(256, 768, 24576);         // rpb 96: 64 + 32
  run(512, 1536, 20480);        // rpb 80 (48-row tiles): 48 + 32
  run(192, 512, 40960);         // two blocks per CU: rpb 80 = 48 + 32
  run(128, 384, 3753659, true);
  if (argc > 1) return 0;
  run(192, 512, 100);
  run(192, 384, 197614);
  run(192, 512, 197614);
  run(192, 640, 197614);
  run(384, 1280, 100);
  run(384, 1280, 49442);
  run(384, 1024, 49442);
  run(384, 768, 49442);
  run(256, 960, 98813);
  run(256, 576, 98813);
  run(256, 768, 98813);
  run(512, 1920, 24753);
  run(512, 1536, 24753);
  run(512, 1152, 24753);
  return 0;
}
