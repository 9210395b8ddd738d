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
  hipLaunchKernelGGL(vibert_embed_kernel, dim3((unsigned)rows), dim3(256), 0, st, a);
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
  hipLaunchKernelGGL(vibert_ln_kernel, dim3((unsigned)rows), dim3(256), 0, st, x, H, g, b, eps);
}

// self-attention of one (sequence, head): K and V of the head in LDS, one query per thread at
// a time; scores / sqrt(d) + the additive padding mask (finfo(f32).min for masked keys, as
// transformers' extended attention mask), softmax (max-subtracted, two passes), context.
// qkv: [B * L][3 H] (q | k | v), ctx: [B * L][H].  L <= 256, head dim D in {16, 32, 64}.
template <int D>
__global__ __launch_bounds__(256) void vibert_attn_kernel(VibertAttnArgs a) {
  __shared__ float sK[256 * D];
  __shared__ float sV[256 * D];
  __shared__ float sM[256];
  const int b = blockIdx.y, h = blockIdx.x, L = a.L, H = a.H;
  const long base = (long)b * L;
  for (int i = threadIdx.x; i < L * D; i += 256) {
    const int j = i / D, d = i % D;
    const float* row = a.qkv + (base + j) * 3 * H;
    sK[i] = row[H + h * D + d];
    sV[i] = row[2 * H + h * D + d];
  }
  for (int j = threadIdx.x; j < L; j += 256)
    sM[j] = a.mask[base + j] ? 0.f : -3.4028234663852886e38f;
  __syncthreads();
  const float scale = a.scale;
  for (int qi = threadIdx.x; qi < L; qi += 256) {
    float q[D];
    const float* qr = a.qkv + (base + qi) * 3 * H + h * D;
#pragma unroll
    for (int d = 0; d < D; ++d) q[d] = qr[d];
    float mx = -INFINITY;
    for (int j = 0; j < L; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s = fmaf(q[d], sK[j * D + d], s);
      mx = fmaxf(mx, s * scale + sM[j]);
    }
    float sum = 0.f, o[D];
#pragma unroll
    for (int d = 0; d < D; ++d) o[d] = 0.f;
    for (int j = 0; j < L; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) s = fmaf(q[d], sK[j * D + d], s);
      const float p = __expf(s * scale + sM[j] - mx);
      sum += p;
#pragma unroll
      for (int d = 0; d < D; ++d) o[d] = fmaf(p, sV[j * D + d], o[d]);
    }
    const float inv = 1.f / sum;
    float* out = a.ctx + (base + qi) * H + h * D;
#pragma unroll
    for (int d = 0; d < D; ++d) out[d] = o[d] * inv;
  }
}

void launch_vibert_attention(const VibertAttnArgs& a, int B, int heads, hipStream_t st) {
  const int D = heads > 0 ? a.H / heads : 0;
  ZASR_REQUIRE(a.L <= 256 && a.H == heads * D && (D == 16 || D == 32 || D == 64),
               "ViBERT attention: L <= 256, head dim 16, 32 or 64");
  if (B <= 0) return;
  if (D == 64)
    hipLaunchKernelGGL(vibert_attn_kernel<64>, dim3(heads, B), dim3(256), 0, st, a);
  else if (D == 32)
    hipLaunchKernelGGL(vibert_attn_kernel<32>, dim3(heads, B), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(vibert_attn_kernel<16>, dim3(heads, B), dim3(256), 0, st, a);
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
  hipLaunchKernelGGL(vibert_gather_kernel, dim3((unsigned)(B * W)), dim3(256), 0, st, x, offsets,
                     L, W, H, g);
}

}  // namespace zasr
