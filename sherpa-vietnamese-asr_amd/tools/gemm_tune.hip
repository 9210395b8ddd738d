// Tile-shape sweep of the encoder projection GEMMs (development tool, not part of libzasr):
// every bf16-mode enc_gemm shape of the 68M bench step (bench.py --shape-table) through every
// register-staged tile (launch_h) and the LDS-DMA kernel (launch_glds), mean of 10 launches
// after 2 warm-ups.  All variants accumulate each output over the same 32-deep K slabs in the
// same MFMA order, so their results are bit-identical (checked here against the default
// launch on 4096 sampled outputs): the choice is a pure speed decision.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o gemm_tune gemm_tune.hip
#include "../csrc/gemm.hip"

#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

using namespace zasr;

struct Shape {
  int M, K, N;
  bool a16, c16;
  int epi;
};

static float* dA;
static __bf16 *dA16, *dB, *dC16, *dRef16;
static float *dC, *dRef, *dbias;

struct SweepResult { float def_us = 0.f, best_us = 1e30f; const char* best = ""; };

template <typename TA, typename TC, int EPI>
static SweepResult sweep(const Shape& s) {
  SweepResult res;
  GemmParams p{};
  p.A = std::is_same<TA, float>::value ? dA : reinterpret_cast<const float*>(dA16);
  p.lda = s.K;
  p.sbk = 1;
  p.sbn = s.K;
  p.C = std::is_same<TC, float>::value ? dC : reinterpret_cast<float*>(dC16);
  p.ldc = s.N;
  p.bias = dbias;
  p.M = s.M;
  p.N = s.N;
  p.K = s.K;
  p.alpha = 1.f;
  p.max_M = s.M;
  const size_t cbytes = (size_t)s.M * s.N * sizeof(TC);
  void* ref = std::is_same<TC, float>::value ? (void*)dRef : (void*)dRef16;
  // reference output of the default launch (RESADD: C starts at zero for the check)
  hipMemset(p.C, 0, cbytes);
  launch_bk_h<ALOAD_DENSE, EPI, TA, TC>(p, dB, 0);
  hipMemcpy(ref, p.C, cbytes, hipMemcpyDeviceToDevice);
  std::vector<std::pair<const char*, std::function<void()>>> vars = {
      {"default", [&] { launch_bk_h<ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"64x64", [&] { launch_h<64, 64, 32, 2, 2, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"64x128", [&] { launch_h<64, 128, 32, 2, 2, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"128x64", [&] { launch_h<128, 64, 32, 2, 2, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"128x128", [&] { launch_h<128, 128, 32, 2, 2, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"128x256", [&] { launch_h<128, 256, 32, 2, 4, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"256x128", [&] { launch_h<256, 128, 32, 4, 2, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"128x32", [&] { launch_h<128, 32, 32, 4, 1, ALOAD_DENSE, EPI, TA, TC>(p, dB, 0); }},
      {"glds3_192", [&] {
         const int tn = cdiv(p.N, 192), tm = cdiv(p.M, 128);
         hipLaunchKernelGGL((gemm_glds_kernel<3, EPI, TA, TC, 192, false>), dim3(tn * tm), dim3(256), 0, 0, p, dB, tn);
       }},
      {"glds4_192", [&] {
         const int tn = cdiv(p.N, 192), tm = cdiv(p.M, 128);
         hipLaunchKernelGGL((gemm_glds_kernel<4, EPI, TA, TC, 192, false>), dim3(tn * tm), dim3(256), 0, 0, p, dB, tn);
       }},
      {"glds3", [&] { launch_glds<3, EPI, TA, TC>(p, dB, 0); }},
      {"glds4", [&] { launch_glds<4, EPI, TA, TC>(p, dB, 0); }},
  };
  // hash of 512 sampled outputs of the default launch (compares builds, e.g. ZASR_GEMM_AQ)
  unsigned long long hsh = 1469598103934665603ull;
  {
    hipDeviceSynchronize();
    std::mt19937 r2(s.M ^ (s.N << 8) ^ (s.K << 16));
    const size_t esz = std::is_same<TC, float>::value ? 4 : 2;
    for (int q = 0; q < 512; ++q) {
      const size_t idx = (size_t)r2() % ((size_t)s.M * s.N);
      unsigned int bits = 0;
      hipMemcpy(&bits, (const char*)ref + idx * esz, esz, hipMemcpyDeviceToHost);
      hsh = (hsh ^ bits) * 1099511628211ull;
    }
  }
  printf("M=%6d K=%5d N=%5d a%s c%s epi%d h=%016llx:", s.M, s.K, s.N, s.a16 ? "16" : "32",
         s.c16 ? "16" : "32", EPI, hsh);
  std::mt19937 rng(7);
  for (auto& v : vars) {
    if (!strncmp(v.first, "glds", 4) && (s.K % 32 != 0 || s.K < 128)) continue;
    if (strstr(v.first, "_192") && s.N % 192 != 0) continue;
    hipMemset(p.C, 0, cbytes);
    v.second();
    hipDeviceSynchronize();
    // bit-identical check on sampled outputs
    std::vector<unsigned short> a(4096), b(4096);
    std::vector<float> af(4096), bf(4096);
    bool same = true;
    for (int q = 0; q < 4096 && same; ++q) {
      const size_t idx = ((size_t)rng() * 2654435761u) % ((size_t)s.M * s.N);
      if (std::is_same<TC, float>::value) {
        hipMemcpy(&af[q], dC + idx, 4, hipMemcpyDeviceToHost);
        hipMemcpy(&bf[q], dRef + idx, 4, hipMemcpyDeviceToHost);
        same = memcmp(&af[q], &bf[q], 4) == 0;
      } else {
        hipMemcpy(&a[q], dC16 + idx, 2, hipMemcpyDeviceToHost);
        hipMemcpy(&b[q], dRef16 + idx, 2, hipMemcpyDeviceToHost);
        same = a[q] == b[q];
      }
      if (q >= 256) break;  // 256 samples keep the sweep short
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    v.second();
    v.second();
    hipEventRecord(e0, 0);
    for (int r = 0; r < 10; ++r) v.second();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("  %s %.1f%s", v.first, ms * 100.f, same ? "" : "(DIFF)");
    if (!strcmp(v.first, "default")) res.def_us = ms * 100.f;
    if (same && ms * 100.f < res.best_us) { res.best_us = ms * 100.f; res.best = v.first; }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  printf("\n");
  fflush(stdout);
  return res;
}

// in-projections of the bf16 step (A = the f32 residual stream today) with A read as f32 (as
// now) and as a bf16 image of the same values: default and best tile of each, weighted by the
// launches per step (bench.py --shape-table, profiles/r05/gemm_h3r/shapes_bf16.json)
struct InProj { int M, K, N, epi, launches; };
static int a16_mode() {
  const std::vector<InProj> v = {
      {49442, 384, 768, EPI_GLU, 12},  {98813, 256, 512, EPI_GLU, 8},   {24753, 512, 1024, EPI_GLU, 8},
      {197561, 192, 384, EPI_GLU, 4},  {49442, 384, 864, EPI_NONE, 6},  {98813, 256, 576, EPI_NONE, 4},
      {197561, 192, 432, EPI_NONE, 2}, {24753, 512, 1152, EPI_NONE, 4}, {49442, 384, 272, EPI_NONE, 6},
      {98813, 256, 272, EPI_NONE, 4},  {197561, 192, 272, EPI_NONE, 2}, {24753, 512, 544, EPI_NONE, 4},
      {49442, 384, 48, EPI_NONE, 12},  {98813, 256, 48, EPI_NONE, 8},   {197561, 192, 48, EPI_NONE, 4},
      {24753, 512, 96, EPI_NONE, 8},
  };
  double t32d = 0, t32b = 0, t16d = 0, t16b = 0, wr = 0;
  for (const InProj& q : v) {
    SweepResult r32, r16;
    if (q.epi == EPI_GLU) {
      r32 = sweep<float, __bf16, EPI_GLU>({q.M, q.K, q.N, false, true, EPI_GLU});
      r16 = sweep<__bf16, __bf16, EPI_GLU>({q.M, q.K, q.N, true, true, EPI_GLU});
    } else {
      r32 = sweep<float, __bf16, EPI_NONE>({q.M, q.K, q.N, false, true, EPI_NONE});
      r16 = sweep<__bf16, __bf16, EPI_NONE>({q.M, q.K, q.N, true, true, EPI_NONE});
    }
    printf("  => M %d K %d N %d epi %d x%d: f32-A default %.1f best %.1f (%s) | bf16-A default %.1f best %.1f (%s)\n",
           q.M, q.K, q.N, q.epi, q.launches, r32.def_us, r32.best_us, r32.best, r16.def_us, r16.best_us, r16.best);
    t32d += q.launches * r32.def_us; t32b += q.launches * r32.best_us;
    t16d += q.launches * r16.def_us; t16b += q.launches * r16.best_us;
    wr += q.launches * (double)q.M * q.K * 2;  // the producer's extra bf16 image write
  }
  printf("per step: f32-A default %.3f ms best %.3f ms | bf16-A default %.3f ms best %.3f ms | "
         "producer bf16 image writes %.1f MB (%.3f ms at 5 TB/s)\n",
         t32d / 1e3, t32b / 1e3, t16d / 1e3, t16b / 1e3, wr / 1e6, wr / 5e12 * 1e3);
  return 0;
}

int main(int argc, char** argv) {
  // bench.py --shape-table, bf16 mode, 68M, 1 h per step (profiles/r03/ffn_w2sets/)
  std::vector<Shape> shapes = {
      {49442, 384, 768, false, true, EPI_NONE},   {49442, 384, 384, true, false, EPI_RESADD},
      {98813, 256, 512, false, true, EPI_NONE},   {98813, 256, 256, true, false, EPI_RESADD},
      {197561, 2432, 192, true, false, EPI_NONE}, {49442, 384, 864, false, true, EPI_NONE},
      {49442, 48, 384, true, false, EPI_RESADD},  {197561, 192, 384, false, true, EPI_NONE},
      {24753, 512, 1024, false, true, EPI_NONE},  {197561, 192, 192, true, false, EPI_RESADD},
      {49442, 288, 384, true, false, EPI_RESADD}, {98813, 48, 256, true, false, EPI_RESADD},
      {24753, 512, 512, true, false, EPI_RESADD}, {98813, 256, 576, false, true, EPI_NONE},
      {197561, 192, 272, false, true, EPI_NONE},  {49442, 384, 272, false, true, EPI_NONE},
      {197561, 48, 192, true, false, EPI_RESADD}, {49442, 384, 48, false, true, EPI_NONE},
      {98813, 256, 272, false, true, EPI_NONE},   {98813, 192, 256, true, false, EPI_RESADD},
      {197561, 192, 432, false, true, EPI_NONE},  {24753, 512, 1152, false, true, EPI_NONE},
      {98813, 256, 48, false, true, EPI_NONE},    {24753, 96, 512, true, false, EPI_RESADD},
      {24753, 512, 544, false, true, EPI_NONE},   {197561, 144, 192, true, false, EPI_RESADD},
      {24753, 512, 96, false, true, EPI_NONE},    {98813, 512, 512, false, false, EPI_NONE},
      {24753, 384, 512, true, false, EPI_RESADD}, {197561, 192, 48, false, true, EPI_NONE},
  };
  size_t maxA = 0, maxC = 0, maxB = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
    maxB = std::max(maxB, (size_t)s.N * s.K);
  }
  hipMalloc(&dA, maxA * 4);
  hipMalloc(&dA16, maxA * 2);
  hipMalloc(&dC, maxC * 4);
  hipMalloc(&dC16, maxC * 2);
  hipMalloc(&dRef, maxC * 4);
  hipMalloc(&dRef16, maxC * 2);
  hipMalloc(&dB, maxB * 2);
  hipMalloc(&dbias, 4096 * 4);
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<float> hA(maxA), hbias(4096);
  std::vector<__bf16> hA16(maxA), hB16(maxB);
  for (size_t i = 0; i < maxA; ++i) {
    hA[i] = nd(rng);
    hA16[i] = (__bf16)hA[i];
  }
  for (auto& x : hB16) x = (__bf16)(nd(rng) * 0.08f);
  for (auto& x : hbias) x = nd(rng) * 0.1f;
  hipMemcpy(dA, hA.data(), maxA * 4, hipMemcpyHostToDevice);
  hipMemcpy(dA16, hA16.data(), maxA * 2, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB16.data(), maxB * 2, hipMemcpyHostToDevice);
  hipMemcpy(dbias, hbias.data(), 4096 * 4, hipMemcpyHostToDevice);
  if (argc > 1 && !strcmp(argv[1], "a16")) return a16_mode();
  for (auto& s : shapes) {
    if (!s.a16 && s.c16 && s.epi == EPI_NONE) sweep<float, __bf16, EPI_NONE>(s);
    else if (s.a16 && !s.c16 && s.epi == EPI_RESADD) sweep<__bf16, float, EPI_RESADD>(s);
    else if (s.a16 && !s.c16 && s.epi == EPI_NONE) sweep<__bf16, float, EPI_NONE>(s);
    else if (!s.a16 && !s.c16 && s.epi == EPI_NONE) sweep<float, float, EPI_NONE>(s);
  }
  return 0;
}
