// Fused Zipformer2 FeedforwardModule in the bf16 mode (icefall zipformer.py, 3P; inside the
// reference's exported encoder, core/asr_engine.py:1045-1049):
//
//   X += W2 SwooshL(W1 X + b1) + b2        X: [R][D] f32 (residual stream), W1 [F][D], W2 [D][F]
//
// The hidden activation (F = 3/4 ff .. 5/4 ff wide) never leaves the CU: one wave owns 32
// tokens (the MFMA column = lane), and for every 32-unit hidden chunk
//   H^T = W1_c X^T           v_mfma_f32_32x32x16_bf16, X^T fragments held in registers
//   H^T <- bf16(SwooshL(H^T + b1_c))   in registers
//   O^T += W2_c H^T          the H^T accumulator registers ARE the B operand (k order
//                            permuted: element j of lane half h at k-step s is hidden row
//                            16 s + 8 (j >> 2) + 4 h + (j & 3)); W2_c is staged in LDS in
//                            that order, so its A fragment is one 16-byte LDS read
// Weight chunks (W1_c [32][D], W2_c [D][32], b1_c) are staged in LDS once per block for its
// 4 waves (128 tokens), double-buffered: the next chunk's global loads are in flight while the
// current chunk computes.  Epilogue: X[token][d] += O^T + b2 (f32 read-modify-write).
// Bytes per token: D * 4 read + D * 4 written; the 2 F D bf16 weight bytes are L2-resident.
#include "common.h"
#include "kernels.h"

namespace zasr {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kTok = 128;  // tokens per block (4 waves x 32)
constexpr int kW2Ld = 40;  // W2 chunk row stride (bf16): 80 B

// slot of hidden index k (0..31) in a permuted W2 chunk row: swap bits 2 and 3
__device__ __forceinline__ int w2_slot(int k) { return (k & 0x13) | ((k & 4) << 1) | ((k & 8) >> 1); }

}  // namespace

template <int D>
__global__ __launch_bounds__(256, (D <= 192 ? 2 : 1)) void ffn_fused_kernel(float* __restrict__ X, int R, int F,
                                                           const __bf16* __restrict__ W1,
                                                           const float* __restrict__ b1,
                                                           const __bf16* __restrict__ W2,
                                                           const float* __restrict__ b2,
                                                           const float* __restrict__ byp_orig,
                                                           const float* __restrict__ byp_scale) {
  constexpr int KS = D / 16;     // k-steps of the first product
  constexpr int OT = D / 32;     // output row tiles of the second
  constexpr int W1LD = D + 8;    // W1 chunk row stride (bf16): odd multiple of 16 B
  constexpr int W1P = 32 * D / 8;  // 16-byte pieces of a W1 chunk
  constexpr int W2P = D * 4;       // 16-byte pieces of a W2 chunk (D rows x 64 B)
  constexpr int P1 = (W1P + 255) / 256, P2 = (W2P + 255) / 256;
  __shared__ __attribute__((aligned(16))) __bf16 sW1[2][32 * W1LD];
  __shared__ __attribute__((aligned(16))) __bf16 sW2[2][D * kW2Ld];
  __shared__ float sB1[2][32];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int col = lane & 31, h2 = lane >> 5;
  const int tok = blockIdx.x * kTok + wid * 32 + col;
  const int tokc = tok < R ? tok : R - 1;
  const int nch = (F + 31) / 32;

  // ---- chunk staging (global -> registers -> LDS) ----
  bf16x8 g1[P1], g2[P2];
  float gb = 0.f;
  auto gload = [&](int c) {
#pragma unroll
    for (int i = 0; i < P1; ++i) {
      const int e = tid + 256 * i < W1P ? tid + 256 * i : W1P - 1;  // clamped, unconditional
      const int row = e / (D / 8), k8 = e - row * (D / 8);
      int hr = c * 32 + row;
      hr = hr < F ? hr : F - 1;  // rows past F: any finite value (their W2 columns are 0)
      g1[i] = *reinterpret_cast<const bf16x8*>(W1 + (long)hr * D + 8 * k8);
    }
#pragma unroll
    for (int i = 0; i < P2; ++i) {
      const int e = tid + 256 * i < W2P ? tid + 256 * i : W2P - 1;
      const int row = e >> 2, q = e & 3;
      const int k0 = c * 32 + 8 * q;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(W2 + (long)row * F + (k0 < F ? k0 : 0));
      if (k0 >= F) {
#pragma unroll
        for (int t = 0; t < 8; ++t) v[t] = (__bf16)0.f;
      }
      g2[i] = v;
    }
    // unconditional (clamped): a guarded load becomes a branch whose vmcnt(0) would wait
    // for the weight loads just issued
    const int bi = c * 32 + (tid & 31);
    const float bv = b1[bi < F ? bi : F - 1];
    gb = bi < F ? bv : 0.f;
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < P1; ++i) {
      const int e = tid + 256 * i;
      if (e < W1P) {
        const int row = e / (D / 8), k8 = e - row * (D / 8);
        *reinterpret_cast<bf16x8*>(&sW1[buf][row * W1LD + 8 * k8]) = g1[i];
      }
    }
#pragma unroll
    for (int i = 0; i < P2; ++i) {
      const int e = tid + 256 * i;
      if (e >= W2P) break;
      const int row = e >> 2, q = e & 3;
      // k = 8 q + m: m = 0..3 -> slot w2_slot(8q), m = 4..7 -> w2_slot(8q + 4)
      bf16x4 lo, hi;
      lo[0] = g2[i][0]; lo[1] = g2[i][1]; lo[2] = g2[i][2]; lo[3] = g2[i][3];
      hi[0] = g2[i][4]; hi[1] = g2[i][5]; hi[2] = g2[i][6]; hi[3] = g2[i][7];
      *reinterpret_cast<bf16x4*>(&sW2[buf][row * kW2Ld + w2_slot(8 * q)]) = lo;
      *reinterpret_cast<bf16x4*>(&sW2[buf][row * kW2Ld + w2_slot(8 * q + 4)]) = hi;
    }
    if (tid < 32) sB1[buf][tid] = gb;
  };

  gload(0);
  // ---- this lane's token row as X^T fragments: element j of k-step s = X[tok][16 s + 8 h2 + j] ----
  bf16x8 xf[KS];
  {
    const float* xr = X + (long)tokc * D + 8 * h2;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(xr + 16 * s);
      const float4 b = *reinterpret_cast<const float4*>(xr + 16 * s + 4);
      xf[s][0] = (__bf16)a.x; xf[s][1] = (__bf16)a.y; xf[s][2] = (__bf16)a.z; xf[s][3] = (__bf16)a.w;
      xf[s][4] = (__bf16)b.x; xf[s][5] = (__bf16)b.y; xf[s][6] = (__bf16)b.z; xf[s][7] = (__bf16)b.w;
    }
  }
  sstore(0);
  __syncthreads();

  f32x16 o[OT];
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) o[t][r] = 0.f;

  for (int c = 0; c < nch; ++c) {
    const int cur = c & 1;
    if (c + 1 < nch) gload(c + 1);
    // H^T = W1_c X^T: rows = hidden units (registers), cols = tokens (lanes)
    f32x16 hacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) hacc[r] = 0.f;
    const __bf16* w1 = &sW1[cur][col * W1LD + 8 * h2];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      hacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w1 + 16 * s),
                                                     xf[s], hacc, 0, 0, 0);
    // + b1, SwooshL, bf16: the two k-step fragments of the second product
    bf16x8 pf[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int hrow = (r & 3) + 8 * (r >> 2) + 4 * h2;
      pf[r >> 3][r & 7] = (__bf16)swooshl_fast(hacc[r] + sB1[cur][hrow]);
    }
    // O^T += W2_c H^T: rows = output channels t*32 + col (A fragment from the permuted chunk)
#pragma unroll
    for (int t = 0; t < OT; ++t) {
      const __bf16* w2 = &sW2[cur][(t * 32 + col) * kW2Ld + 8 * h2];
      o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w2), pf[0], o[t], 0, 0, 0);
      o[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(w2 + 16), pf[1], o[t], 0, 0, 0);
    }
    if (c + 1 < nch) sstore(cur ^ 1);
    __syncthreads();
  }

  // ---- X[tok][d] += O^T + b2: lane's token, channels t*32 + 8 g + 4 h2 + (0..3) ----
  if (tok >= R) return;
  float* xr = X + (long)tok * D;
#pragma unroll
  for (int t = 0; t < OT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int ch = t * 32 + 8 * g + 4 * h2;
      const float4 bb = *reinterpret_cast<const float4*>(b2 + ch);
      float4 v = *reinterpret_cast<const float4*>(xr + ch);
      v.x += o[t][4 * g + 0] + bb.x;
      v.y += o[t][4 * g + 1] + bb.y;
      v.z += o[t][4 * g + 2] + bb.z;
      v.w += o[t][4 * g + 3] + bb.w;
      if (byp_orig != nullptr) {  // bypass_mid folded in (launch_bypass's formula)
        const float4 b0 = *reinterpret_cast<const float4*>(byp_orig + (long)tok * D + ch);
        const float4 k = *reinterpret_cast<const float4*>(byp_scale + ch);
        v.x = b0.x + (v.x - b0.x) * k.x;
        v.y = b0.y + (v.y - b0.y) * k.y;
        v.z = b0.z + (v.z - b0.z) * k.z;
        v.w = b0.w + (v.w - b0.w) * k.w;
      }
      *reinterpret_cast<float4*>(xr + ch) = v;
    }
}

// D = 256 compiles to one wave per SIMD (384 registers) and measured slower than the two
// GEMMs (tools/ffn_lab.hip): fused only up to 192
bool ffn_fused_supported(int D) { return D == 64 || D == 96 || D == 128 || D == 192; }

void launch_ffn_fused(float* X, int R, int D, int F, const void* W1, const float* b1,
                      const void* W2, const float* b2, hipStream_t st, const float* byp_orig,
                      const float* byp_scale) {
  if (R <= 0) return;
  ZASR_REQUIRE(ffn_fused_supported(D), "ffn_fused: unsupported model dim");
  ZASR_REQUIRE(F % 8 == 0, "ffn_fused: feed-forward dim must be a multiple of 8");
  const dim3 grid(cdiv(R, kTok));
  const __bf16* w1 = reinterpret_cast<const __bf16*>(W1);
  const __bf16* w2 = reinterpret_cast<const __bf16*>(W2);
#define ZASR_FFN(DV) hipLaunchKernelGGL(ffn_fused_kernel<DV>, grid, dim3(256), 0, st, X, R, F, w1, b1, w2, b2, byp_orig, byp_scale)
  switch (D) {
    case 64: ZASR_FFN(64); break;
    case 96: ZASR_FFN(96); break;
    case 128: ZASR_FFN(128); break;
    case 192: ZASR_FFN(192); break;
    default: ZASR_FFN(256); break;
  }
#undef ZASR_FFN
}

}  // namespace zasr
