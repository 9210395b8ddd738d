// ViBERT-capu (BERT encoder + Seq2Labels heads) kernels other than the projections, which run
// on the exact-f32 MFMA GEMM (gemm.hip: fused QKV, attention output + residual, FFN with the
// erf GELU epilogue + residual, the two label heads).  SURVEY §8f row 3; the graph is the
// reference's convert_onnx/export_vibert_onnx.py Seq2LabelsModel run at core/gec_model.py:366-412.
#include "common.h"
#include "kernels.h"

namespace zasr {

namespace {
// block-wide sum of a double over 256 threads
__device__ double block_sum256(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// LayerNorm of one row held as up to 4 values per thread (H <= 1024), in place into y
__device__ void layer_norm_row(float* v, int H, const float* g, const float* b, float eps,
                               float* y, double* red) {
  const int tid = threadIdx.x;
  double s = 0.0;
  for (int k = 0; k < 4; ++k)
    if (tid + 256 * k < H) s += v[k];
  const double mean = block_sum256(s, red) / H;
  double q = 0.0;
  for (int k = 0; k < 4; ++k)
    if (tid + 256 * k < H) {
      const double d = v[k] - mean;
      q += d * d;
    }
  const double var = block_sum256(q, red) / H;
  const float rstd = (float)(1.0 / sqrt(var + eps));
  for (int k = 0; k < 4; ++k) {
    const int c = tid + 256 * k;
    if (c < H) y[c] = ((v[k] - (float)mean) * rstd) * g[c] + b[c];
  }
}
}  // namespace

// embeddings: x[r] = LN(word[ids[r]] + pos[r % L] + type[tt[r]]), one block per token row
__global__ __launch_bounds__(256) void vibert_embed_kernel(VibertEmbedArgs a) {
  __shared__ double red[4];
  const long r = blockIdx.x;
  const int l = (int)(r % a.L);
  const long id = a.ids[r], tt = a.tt[r];
  float v[4];
  for (int k = 0; k < 4; ++k) {
    const int c = threadIdx.x + 256 * k;
    v[k] = c < a.H ? a.word[id * a.H + c] + a.pos[(long)l * a.H + c] + a.type[tt * a.H + c] : 0.f;
  }
  layer_norm_row(v, a.H, a.ln_g, a.ln_b, a.eps, a.x + r * a.H, red);
}

void launch_vibert_embed(const VibertEmbedArgs& a, long rows, hipStream_t st) {
  ZASR_REQUIRE(a.H <= 1024, "ViBERT: hidden size must be <= 1024");
  if (rows <= 0) return;
  ZASR_LAUNCH(vibert_embed_kernel, dim3((unsigned)rows), dim3(256), 0, st, a);
}

__global__ __launch_bounds__(256) void vibert_ln_kernel(float* x, int H, const float* g,
                                                        const float* b, float eps) {
  __shared__ double red[4];
  float* row = x + (long)blockIdx.x * H;
  float v[4];
  for (int k = 0; k < 4; ++k) {
    const int c = threadIdx.x + 256 * k;
    v[k] = c < H ? row[c] : 0.f;
  }
  layer_norm_row(v, H, g, b, eps, row, red);
}

void launch_vibert_layernorm(float* x, long rows, int H, const float* g, const float* b, float eps,
                             hipStream_t st) {
  ZASR_REQUIRE(H <= 1024, "ViBERT: hidden size must be <= 1024");
  if (rows <= 0) return;
  ZASR_LAUNCH(vibert_ln_kernel, dim3((unsigned)rows), dim3(256), 0, st, x, H, g, b, eps);
}

// self-attention of one (sequence, head): K (row stride D + 1: conflict-free per-lane rows)
// and V of the head in LDS, sized to L; each of the 4 waves takes queries qi = wave, wave + 4,
// ...: lanes own keys j = lane + 64 c for the scores (q broadcast from LDS; the same fmaf
// chain over d as a per-query loop), a wave max, p_j = exp(s_j * scale + mask_j - max) to a
// per-wave LDS row, then lane d accumulates the context over j in ascending order together
// with the sum of p (sequential, as a per-query loop would).  Scores / sqrt(d) + the additive
// padding mask (finfo(f32).min for masked keys, as transformers' extended attention mask).
// qkv: [B * L][3 H] (q | k | v), ctx: [B * L][H].  L <= 256, head dim D in {16, 32, 64}.
template <int D>
__global__ __launch_bounds__(256) void vibert_attn_kernel(VibertAttnArgs a) {
  constexpr int KS = D + 1;
  extern __shared__ float smem[];
  const int L = a.L, H = a.H;
  float* sK = smem;             // [L][D + 1]
  float* sV = sK + L * KS;      // [L][D]
  float* sM = sV + L * D;       // [L]
  float* sP = sM + L;           // [4][L]
  float* sQ = sP + 4 * L;       // [4][D]
  const int b = blockIdx.y, h = blockIdx.x;
  const long base = (long)b * L;
  for (int i = threadIdx.x; i < L * D; i += 256) {
    const int j = i / D, d = i - j * D;
    const float* row = a.qkv + (base + j) * 3 * H;
    sK[j * KS + d] = row[H + h * D + d];
    sV[i] = row[2 * H + h * D + d];
  }
  for (int j = threadIdx.x; j < L; j += 256)
    sM[j] = a.mask[base + j] ? 0.f : -3.4028234663852886e38f;
  __syncthreads();
  const float scale = a.scale;
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float* q = sQ + wid * D;
  float* pw = sP + wid * L;
  for (int qi = wid; qi < L; qi += 4) {
    if (lane < D) q[lane] = a.qkv[(base + qi) * 3 * H + h * D + lane];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // q visible to the whole wave
    __builtin_amdgcn_wave_barrier();
    float sc[4];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = lane + 64 * c;
      sc[c] = -INFINITY;
      if (j < L) {
        float s = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) s = fmaf(q[d], sK[j * KS + d], s);
        sc[c] = s * scale + sM[j];
        mx = fmaxf(mx, sc[c]);
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = lane + 64 * c;
      if (j < L) pw[j] = __expf(sc[c] - mx);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (lane < D) {
      float sum = 0.f, o = 0.f;
      for (int j = 0; j < L; ++j) {
        const float p = pw[j];
        sum += p;
        o = fmaf(p, sV[j * D + lane], o);
      }
      a.ctx[(base + qi) * H + h * D + lane] = o * (1.f / sum);
    }
    __builtin_amdgcn_wave_barrier();  // the next query rewrites q and pw
  }
}

static size_t vibert_attn_lds(int L, int D) {
  return sizeof(float) * ((size_t)L * (2 * D + 1) + L + 4 * (size_t)L + 4 * (size_t)D);
}

void launch_vibert_attention(const VibertAttnArgs& a, int B, int heads, hipStream_t st) {
  const int D = heads > 0 ? a.H / heads : 0;
  ZASR_REQUIRE(a.L <= 256 && a.H == heads * D && (D == 16 || D == 32 || D == 64),
               "ViBERT attention: L <= 256, head dim 16, 32 or 64");
  if (B <= 0) return;
  const size_t lds = vibert_attn_lds(a.L, D);
  static bool attr = false;
  if (!attr) {  // up to 138 KB of LDS at L = 256, D = 64
    const int mx = (int)vibert_attn_lds(256, 64);
    ZASR_HIP_CHECK(hipFuncSetAttribute((const void*)vibert_attn_kernel<64>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    ZASR_HIP_CHECK(hipFuncSetAttribute((const void*)vibert_attn_kernel<32>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    ZASR_HIP_CHECK(hipFuncSetAttribute((const void*)vibert_attn_kernel<16>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, mx));
    attr = true;
  }
  if (D == 64)
    ZASR_LAUNCH(vibert_attn_kernel<64>, dim3(heads, B), dim3(256), lds, st, a);
  else if (D == 32)
    ZASR_LAUNCH(vibert_attn_kernel<32>, dim3(heads, B), dim3(256), lds, st, a);
  else
    ZASR_LAUNCH(vibert_attn_kernel<16>, dim3(heads, B), dim3(256), lds, st, a);
}

// g[b * W + w] = x[b * L + offsets[b][w]]
__global__ void vibert_gather_kernel(const float* __restrict__ x, const long* __restrict__ off,
                                     int L, int W, int H, float* __restrict__ g) {
  const long r = blockIdx.x;
  const int b = (int)(r / W);
  const long src = (long)b * L + off[r];
  for (int c = threadIdx.x; c < H; c += blockDim.x) g[r * H + c] = x[src * H + c];
}

void launch_vibert_gather(const float* x, const long* offsets, int B, int L, int W, int H, float* g,
                          hipStream_t st) {
  if (B * W <= 0) return;
  ZASR_LAUNCH(vibert_gather_kernel, dim3((unsigned)(B * W)), dim3(256), 0, st, x, offsets,
                     L, W, H, g);
}

}  // namespace zasr
