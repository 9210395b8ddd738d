// Transducer search on device: modified beam search (greedy = beam 1) with Aho-Corasick
// hotword biasing, restating core/asr_engine.py:1023-1153 and core/hotword_context.py.
//
// Per frame t, two launches:
//   joiner             logits[S*H, V] = W_out J + b                           (:1090-1093)
//   search_step_kernel one block per stream:
//     1. per live hypothesis row: max, second max, sum exp, entropy terms (the reference's
//        f32 numpy log-softmax :1096-1098 and _compute_token_entropy :1159-1181)
//     2. candidates lp = ((logit - max) - log(sum)) + score_h (f32 add of the Python-float
//        score, or the f64 add of an np.float64 score, :1099-1100); global top-k over H*V
//     3. expansion in descending order (:1110-1138): blank keeps the sequence, non-blank
//        appends, hotword delta after top-k (:1127-1131), duplicates of the full token
//        sequence (identified by (length, 64-bit rolling hash)) merge with an f64 log-add;
//        emissions append a node {token, frame, parent, token logp, row stats}
//     4. the next frame's joiner input J[slot] = tanh(enc[s, t + 1] + dec(y[-2], y[-1]))
//        gathered from the decoder-context table (kernels.h, DecTable) -- the reference's
//        dec_sess / dec_cache (:1051-1056, :1072-1088) evaluated once per context at load.
// Without the table (vocabularies too large for it) a third launch, decjoin_kernel,
// recomputes the decoder for every live slot (Embedding -> grouped Conv1d -> ReLU ->
// decoder_proj on MFMA) and writes J.
// All hypothesis state lives in LDS during the step; global memory is written once.
#include "common.h"
#include "gemm_dev.h"
#include "kernels.h"

#include <cstdlib>

namespace zasr {

namespace {

constexpr unsigned long long kHash0 = 0x6a09e667f3bcc908ull;
constexpr int kMaxBeam = 16;

__device__ __forceinline__ unsigned long long hash_push(unsigned long long h, int tok) {
  unsigned long long x = h ^ (0x9e3779b97f4a7c15ull + (unsigned long long)(unsigned)tok +
                              (h << 6) + (h >> 2));
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// f64 log-add; *f64 = 1 when the reference's result type is np.float64 (non-cutoff branch)
__device__ __forceinline__ double log_add(double a, int fa, double b, int fb, int* f64) {
  if (a < b) {
    double t = a;
    a = b;
    b = t;
    int tf = fa;
    fa = fb;
    fb = tf;
  }
  double d = b - a;
  if (d < -36.0) {
    *f64 = fa;
    return a;
  }
  *f64 = 1;
  return a + log1p(exp(d));
}

// candidate order: larger value first, then smaller flat index, as one unsigned 64-bit key
// (order-preserving float bits << 32 | ~index); key 0 = empty
__device__ __forceinline__ unsigned long long make_key(float v, int idx) {
  unsigned u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (unsigned)(~(unsigned)idx);
}
__device__ __forceinline__ float key_val(unsigned long long k) {
  unsigned u = (unsigned)(k >> 32);
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __uint_as_float(u);
}
__device__ __forceinline__ int key_idx(unsigned long long k) { return (int)(~(unsigned)k); }

// relu(grouped conv(E[y2], E[y1])) for 4 channels c..c+3: the conv is linear per tap, so
// tap0[v] = W[:, :, 0] * E[v] and tap1[v] = W[:, :, 1] * E[v] are tabulated at load time
// (Conv1d(D, D, k=2, groups=D/4, bias=False); tap 0 = older token y[-2], tap 1 = y[-1])
__device__ __forceinline__ float4 dec_conv4(const DecoderW& dw, int y2, int y1, int c) {
  const float4 a = *reinterpret_cast<const float4*>(dw.tap0 + (long)y2 * dw.D + c);
  const float4 b = *reinterpret_cast<const float4*>(dw.tap1 + (long)y1 * dw.D + c);
  return make_float4(fmaxf(a.x + b.x, 0.f), fmaxf(a.y + b.y, 0.f), fmaxf(a.z + b.z, 0.f),
                     fmaxf(a.w + b.w, 0.f));
}

// acc += A[32 rows][k in this wave's range] * B[32 cols][k]^T with f32 MFMA 32x32x2.
// A in LDS ([32][lda]), B = one weight row per lane column (K contiguous), read as float4:
// lane half h covers k = kb + 4h + j (j = 0..3).  All of the wave's B loads are issued
// before the MFMAs (kw <= 128, i.e. D <= 512).
template <int NQ>  // NQ = (k per wave) / 8 = D / 32
__device__ __forceinline__ void tile32_splitk(const float* As, int lda, const float* brow,
                                              bool bvalid, int kbeg, f32x16& acc) {
  const int lane = threadIdx.x & 63;
  const int col = lane & 31, h = lane >> 5;
  float4 b[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q)
    b[q] = bvalid ? *reinterpret_cast<const float4*>(brow + kbeg + 8 * q + 4 * h)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const float4 a = *reinterpret_cast<const float4*>(As + col * lda + kbeg + 8 * q + 4 * h);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[q].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[q].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[q].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[q].w, acc, 0, 0, 0);
  }
}

// waves 1..3 hand their partial tiles to wave 0 through LDS (red: [3][16][64])
__device__ __forceinline__ void splitk_reduce(f32x16& acc, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (wid > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wid - 1) * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r)
      acc[r] += red[r * 64 + lane] + red[(16 + r) * 64 + lane] + red[(32 + r) * 64 + lane];
  }
}

// all streams of joiner rows m0 .. m0 + 31 finished (speculative greedy windows)
__device__ __forceinline__ bool tile_done(const int* live_t, const int* live_len, int F, int m0,
                                          int M) {
  if (!live_t) return false;
  const int s0 = m0 / F, s1 = (min(m0 + 32, M) - 1) / F;
  for (int s = s0; s <= s1; ++s)
    if (live_t[s] < live_len[s]) return false;
  return true;
}

// ---- wave reductions on DPP + readlane (no LDS round trips) ----
// The search kernels run one block per stream, one wave per SIMD: every cross-lane step is
// exposed latency.  __shfl_xor lowers to ds_bpermute_b32 (an LDS round trip per step, six per
// reduction); here a 16-lane row reduces in four DPP steps (quad_perm 1-0-3-2, 2-3-0-1,
// row_ror 4, row_ror 8) and the four row results are combined as scalars via v_readlane.
// Max / min / the (max, second max) merge are exact in any order.  The float sum is
// deterministic (every lane gets the same value) but associates differently from a
// butterfly: every search kernel uses this one function, so the frame-by-frame and the
// speculative greedy kernels still agree bit for bit.
constexpr int kDppQuad1 = 0xB1, kDppQuad2 = 0x4E, kDppRor4 = 0x124, kDppRor8 = 0x128;

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<CTRL>(__float_as_int(v)));
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f<kDppQuad1>(v);
  v += dpp_f<kDppQuad2>(v);
  v += dpp_f<kDppRor4>(v);
  v += dpp_f<kDppRor8>(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_min_dpp(float v) {
  v = fminf(v, dpp_f<kDppQuad1>(v));
  v = fminf(v, dpp_f<kDppQuad2>(v));
  v = fminf(v, dpp_f<kDppRor4>(v));
  v = fminf(v, dpp_f<kDppRor8>(v));
  return fminf(fminf(lane_f(v, 0), lane_f(v, 16)), fminf(lane_f(v, 32), lane_f(v, 48)));
}
// (max, second max) over the wave's (m1, m2) pairs
template <int CTRL>
__device__ __forceinline__ void max2_step(float& m1, float& m2, float a1, float a2) {
  const float hi = fmaxf(m1, a1);
  const float lo = fmaxf(fminf(m1, a1), fmaxf(m2, a2));
  m1 = hi;
  m2 = lo;
}
__device__ __forceinline__ void wave_max2_dpp(float& m1, float& m2) {
  max2_step<0>(m1, m2, dpp_f<kDppQuad1>(m1), dpp_f<kDppQuad1>(m2));
  max2_step<0>(m1, m2, dpp_f<kDppQuad2>(m1), dpp_f<kDppQuad2>(m2));
  max2_step<0>(m1, m2, dpp_f<kDppRor4>(m1), dpp_f<kDppRor4>(m2));
  max2_step<0>(m1, m2, dpp_f<kDppRor8>(m1), dpp_f<kDppRor8>(m2));
  float r1 = lane_f(m1, 0), r2 = lane_f(m2, 0);
#pragma unroll
  for (int l = 16; l < 64; l += 16) max2_step<0>(r1, r2, lane_f(m1, l), lane_f(m2, l));
  m1 = r1;
  m2 = r2;
}
__device__ __forceinline__ unsigned long long lane_u64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f<kDppQuad1>(v));
  v = fmaxf(v, dpp_f<kDppQuad2>(v));
  v = fmaxf(v, dpp_f<kDppRor4>(v));
  v = fmaxf(v, dpp_f<kDppRor8>(v));
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
__device__ __forceinline__ unsigned long long shfl_u64(unsigned long long v, int l) {
  const unsigned lo = (unsigned)__shfl((int)(unsigned)v, l);
  const unsigned hi = (unsigned)__shfl((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double shfl_f64(double v, int l) {
  return __longlong_as_double((long long)shfl_u64((unsigned long long)__double_as_longlong(v), l));
}
__device__ __forceinline__ int wave_min_i_dpp(int v) {
  v = min(v, dpp_i<kDppQuad1>(v));
  v = min(v, dpp_i<kDppQuad2>(v));
  v = min(v, dpp_i<kDppRor4>(v));
  v = min(v, dpp_i<kDppRor8>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// tanh(x) = 1 - 2 / (exp(2x) + 1): saturates correctly at +-inf (bf16 joiner input only)
__device__ __forceinline__ float fast_tanh(float x) { return 1.f - 2.f / (__expf(2.f * x) + 1.f); }

}  // namespace

// --------------------------------------------------------------------------------------
__global__ void search_init_kernel(SearchState s, int S, int Hmax) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S * Hmax) return;
  int slot = i % Hmax;
  s.lp[i] = 0.0;
  s.lpf[i] = 0;
  s.hash[i] = kHash0;
  s.len[i] = 2;  // ys = [-1, blank]
  s.y1[i] = 0;
  s.y2[i] = 0;   // max(0, -1)
  s.hw[i] = 0;   // automaton root
  s.node[i] = -1;
  if (slot == 0) {
    s.nh[i / Hmax] = 1;
    s.node_count[i / Hmax] = 0;
  }
}

void launch_search_init(const SearchState& s, int S, int Hmax, hipStream_t st) {
  int n = S * Hmax;
  if (n <= 0) return;
  ZASR_LAUNCH(search_init_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, s, S, Hmax);
}

// --------------------------------------------------------------------------------------
// decoder + joiner input: block = 32 slots x 32 decoder channels, 4 waves split K.
// --------------------------------------------------------------------------------------
template <int NQ>
__global__ __launch_bounds__(256) void decjoin_kernel(DecJoinArgs a) {
  extern __shared__ float smem[];
  const int D = a.dw.D;
  const int lda = D + 4;
  float* As = smem;                // relu(conv(E[y2], E[y1])) rows  [32][D + 4]
  float* red = smem + 32 * lda;    // [3][16][64]
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d4 = D / 4;
  for (int e = tid; e < 32 * d4; e += 256) {
    const int i = e / d4, c4 = e - i * d4;
    const int r = m0 + i;
    const float4 v = (r < a.M) ? dec_conv4(a.dw, a.y2[r], a.y1[r], 4 * c4)
                               : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(As + i * lda + 4 * c4) = v;
  }
  __syncthreads();
  const int n = n0 + (lane & 31);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  tile32_splitk<NQ>(As, lda, a.wp + (long)n * D, true, wid * (D / 4), acc);
  splitk_reduce(acc, red);
  if (wid == 0) {
    const float bp = a.dw.bp[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row >= a.M) continue;
      const int s = row / a.H;
      const float e = a.enc[(long)(a.enc_off[s] + a.t) * D + n];
      const float v = tanhf(e + (acc[r] + bp));
      if (a.j_bf16)
        reinterpret_cast<__bf16*>(a.J)[(long)row * D + n] = (__bf16)v;
      else
        reinterpret_cast<float*>(a.J)[(long)row * D + n] = v;
    }
  }
}

void launch_decjoin(const DecJoinArgs& a, hipStream_t st) {
  if (a.M <= 0) return;
  ZASR_REQUIRE(a.dw.D % 32 == 0 && a.dw.D <= 512, "decoder/joiner dim must be a multiple of 32, <= 512");
  dim3 grid(a.dw.D / 32, cdiv(a.M, 32));
  size_t lds = (32 * (a.dw.D + 4) + 3 * 16 * 64) * sizeof(float);
  switch (a.dw.D / 32) {
    case 2: ZASR_LAUNCH(decjoin_kernel<2>, grid, dim3(256), lds, st, a); break;
    case 4: ZASR_LAUNCH(decjoin_kernel<4>, grid, dim3(256), lds, st, a); break;
    case 8: ZASR_LAUNCH(decjoin_kernel<8>, grid, dim3(256), lds, st, a); break;
    case 16: ZASR_LAUNCH(decjoin_kernel<16>, grid, dim3(256), lds, st, a); break;
    default: throw std::runtime_error("decoder dim must be 64, 128, 256 or 512");
  }
}

// --------------------------------------------------------------------------------------
// decoder-context table: rows r = y2 * V + y1, the decjoin arithmetic (same K split, same
// reduction order) so that table rows equal the per-slot decoder bit for bit.
// --------------------------------------------------------------------------------------
template <int NQ>
__global__ __launch_bounds__(256) void dec_table_kernel(DecoderW dw, const float* __restrict__ wp,
                                                        int V, float* __restrict__ table) {
  extern __shared__ float smem[];
  const int D = dw.D;
  const int lda = D + 4;
  float* As = smem;
  float* red = smem + 32 * lda;
  const long M = (long)V * V;
  const long m0 = (long)blockIdx.x * 32;
  const int n0 = blockIdx.y * 32;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d4 = D / 4;
  for (int e = tid; e < 32 * d4; e += 256) {
    const int i = e / d4, c4 = e - i * d4;
    const long r = m0 + i;
    const float4 v = (r < M) ? dec_conv4(dw, (int)(r / V), (int)(r % V), 4 * c4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(As + i * lda + 4 * c4) = v;
  }
  __syncthreads();
  const int n = n0 + (lane & 31);
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  tile32_splitk<NQ>(As, lda, wp + (long)n * D, true, wid * (D / 4), acc);
  splitk_reduce(acc, red);
  if (wid == 0) {
    const float bp = dw.bp[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const long row = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < M) table[row * D + n] = acc[r] + bp;
    }
  }
}

void launch_dec_table(const DecoderW& dw, const float* wp, int V, float* table, hipStream_t st) {
  ZASR_REQUIRE(dw.D % 32 == 0 && dw.D <= 512, "decoder dim must be a multiple of 32, <= 512");
  const long M = (long)V * V;
  dim3 grid((unsigned)cdivl(M, 32), dw.D / 32);
  size_t lds = (32 * (dw.D + 4) + 3 * 16 * 64) * sizeof(float);
  switch (dw.D / 32) {
    case 2: ZASR_LAUNCH(dec_table_kernel<2>, grid, dim3(256), lds, st, dw, wp, V, table); break;
    case 4: ZASR_LAUNCH(dec_table_kernel<4>, grid, dim3(256), lds, st, dw, wp, V, table); break;
    case 8: ZASR_LAUNCH(dec_table_kernel<8>, grid, dim3(256), lds, st, dw, wp, V, table); break;
    case 16: ZASR_LAUNCH(dec_table_kernel<16>, grid, dim3(256), lds, st, dw, wp, V, table); break;
    default: throw std::runtime_error("decoder dim must be 64, 128, 256 or 512");
  }
}

// --------------------------------------------------------------------------------------
// joiner: logits = W_out J + b; block = 32 rows x 32 vocab columns, 4 waves split K.
// --------------------------------------------------------------------------------------
template <int NQ>
__global__ __launch_bounds__(256) void joiner_kernel(JoinerArgs j) {
  extern __shared__ float smem[];
  const int D = j.D;
  const int lda = D + 4;
  float* As = smem;
  float* red = smem + 32 * lda;
  const int m0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
  if (tile_done(j.live_t, j.live_len, j.live_f, m0, j.M)) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int d4 = D / 4;
  for (int e = tid; e < 32 * d4; e += 256) {
    const int i = e / d4, k4 = e - i * d4;
    const int r = m0 + i;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < j.M) v = reinterpret_cast<const float4*>(j.J + (long)r * D)[k4];
    *reinterpret_cast<float4*>(As + i * lda + 4 * k4) = v;
  }
  __syncthreads();
  const int n = n0 + (lane & 31);
  const bool nv = n < j.V;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  tile32_splitk<NQ>(As, lda, j.W + (long)(nv ? n : 0) * D, nv, wid * (D / 4), acc);
  splitk_reduce(acc, red);
  if (wid == 0 && nv) {
    const float bias = j.bias[n];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (row < j.M) j.out[(long)row * j.V + n] = acc[r] + bias;
    }
  }
}

template <int NP, int FMT = 0>
void launch_joiner_split(const JoinerArgs& j, hipStream_t st);

void launch_joiner(const JoinerArgs& j, hipStream_t st) {
  if (j.M <= 0) return;
  if (j.Wx != nullptr) {  // split-bf16 modes (defined below)
    ZASR_REQUIRE(j.pieces == 2 || j.pieces == 3 || j.pieces == kPiecesF16,
                 "joiner: pieces must be 2, 3 or kPiecesF16");
    if (j.pieces == 2)
      launch_joiner_split<2>(j, st);
    else if (j.pieces == 3)
      launch_joiner_split<3>(j, st);
    else
      launch_joiner_split<2, 1>(j, st);
    return;
  }
  ZASR_REQUIRE(j.D % 32 == 0 && j.D <= 512, "joiner_dim must be a multiple of 32, <= 512");
  dim3 grid(cdiv(j.V, 32), cdiv(j.M, 32));
  size_t lds = (32 * (j.D + 4) + 3 * 16 * 64) * sizeof(float);
  switch (j.D / 32) {
    case 2: ZASR_LAUNCH(joiner_kernel<2>, grid, dim3(256), lds, st, j); break;
    case 4: ZASR_LAUNCH(joiner_kernel<4>, grid, dim3(256), lds, st, j); break;
    case 8: ZASR_LAUNCH(joiner_kernel<8>, grid, dim3(256), lds, st, j); break;
    case 16: ZASR_LAUNCH(joiner_kernel<16>, grid, dim3(256), lds, st, j); break;
    default: throw std::runtime_error("joiner dim must be 64, 128, 256 or 512");
  }
}

// --------------------------------------------------------------------------------------
// bf16 joiner: logits = W_out J + b with J, W_out in bf16 (v_mfma_f32_32x32x16_bf16, f32
// accumulate).  Block = 32 rows x 32 vocab columns; the 4 waves split K (each issues all of
// its J / W_out fragment loads at once: one memory round trip), partial tiles reduced
// through LDS.  Grid = V/32 x M/32 blocks (>= 250 at greedy batch 120: the whole chip).
// --------------------------------------------------------------------------------------
template <int NK>  // NK = D / 64 k16-steps per wave
__global__ __launch_bounds__(256) void joiner_bf16_kernel(JoinerBf16Args j) {
  __shared__ float red[3 * 16 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32;
  if (tile_done(j.live_t, j.live_len, j.live_f, m0, j.M)) return;
  const int n = blockIdx.x * 32 + col;
  const bool nv = n < j.V;
  const int D = j.D;
  const int ar = m0 + col < j.M ? m0 + col : j.M - 1;
  const int kb = wid * (D / 4) + 8 * h;
  const __bf16* arow = j.J + (long)ar * D + kb;
  const __bf16* brow = j.W + (long)(nv ? n : 0) * D + kb;
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
  splitk_reduce(acc, red);
  if (wid != 0 || !nv) return;
  const float bias = j.bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < j.M) j.out[(long)row * j.V + n] = acc[r] + bias;
  }
}

void launch_joiner_bf16(const JoinerBf16Args& j, hipStream_t st) {
  if (j.M <= 0) return;
  dim3 grid(cdiv(j.V, 32), cdiv(j.M, 32));
  switch (j.D) {
    case 64: ZASR_LAUNCH(joiner_bf16_kernel<1>, grid, dim3(256), 0, st, j); break;
    case 128: ZASR_LAUNCH(joiner_bf16_kernel<2>, grid, dim3(256), 0, st, j); break;
    case 256: ZASR_LAUNCH(joiner_bf16_kernel<4>, grid, dim3(256), 0, st, j); break;
    case 512: ZASR_LAUNCH(joiner_bf16_kernel<8>, grid, dim3(256), 0, st, j); break;
    default: throw std::runtime_error("joiner dim must be 64, 128, 256 or 512");
  }
}

// --------------------------------------------------------------------------------------
// split-bf16 joiner (the bf16x3 / bf16x6 modes): J f32 split into NP bf16 pieces as it is
// loaded, W_out pre-split (piece t at Wx + t V D); the products of the pieces (3 / 6 MFMAs per
// k16 step) accumulate in f32 -- near-f32 / f32-quality logits at bf16 MFMA rates.  Same
// block / wave / split-K structure as joiner_bf16_kernel.
// --------------------------------------------------------------------------------------
template <int NK, int NP, int FMT = 0>
__global__ __launch_bounds__(256) void joiner_split_kernel(JoinerArgs j) {
  __shared__ float red[3 * 16 * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int col = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * 32;
  if (tile_done(j.live_t, j.live_len, j.live_f, m0, j.M)) return;
  const int n = blockIdx.x * 32 + col;
  const bool nv = n < j.V;
  const int D = j.D;
  const long blo = (long)j.V * D;
  const int ar = m0 + col < j.M ? m0 + col : j.M - 1;
  const int kb = wid * (D / 4) + 8 * h;
  const float* arow = j.J + (long)ar * D + kb;
  const __bf16* brow = j.Wx + (long)(nv ? n : 0) * D + kb;
  float4 x0[NK], x1[NK];
  bf16x8 b[NP][NK];
#pragma unroll
  for (int q = 0; q < NK; ++q) {
    x0[q] = *reinterpret_cast<const float4*>(arow + 16 * q);
    x1[q] = *reinterpret_cast<const float4*>(arow + 16 * q + 4);
#pragma unroll
    for (int t = 0; t < NP; ++t) b[t][q] = *reinterpret_cast<const bf16x8*>(brow + t * blo + 16 * q);
  }
  f32x16 acc, accl;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = accl[r] = 0.f;
#pragma unroll
  for (int q = 0; q < NK; ++q) {
    const float v[8] = {x0[q].x, x0[q].y, x0[q].z, x0[q].w, x1[q].x, x1[q].y, x1[q].z, x1[q].w};
    bf16x8 ap[NP], bp[NP];
    split_fx<FMT, NP>(v, ap);
#pragma unroll
    for (int t = 0; t < NP; ++t) bp[t] = b[t][q];
    if constexpr (FMT == 1) {
      mfma_h3(ap, bp, acc, accl);
    } else {
      acc = mfma_split<NP>(ap, bp, acc);
    }
  }
  if constexpr (FMT == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += accl[r] * kF16LoInv;
  }
  splitk_reduce(acc, red);
  if (wid != 0 || !nv) return;
  const float bias = j.bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < j.M) j.out[(long)row * j.V + n] = acc[r] + bias;
  }
}

template <int NP, int FMT>
void launch_joiner_split(const JoinerArgs& j, hipStream_t st) {
  dim3 grid(cdiv(j.V, 32), cdiv(j.M, 32));
  switch (j.D) {
    case 64: ZASR_LAUNCH((joiner_split_kernel<1, NP, FMT>), grid, dim3(256), 0, st, j); break;
    case 128: ZASR_LAUNCH((joiner_split_kernel<2, NP, FMT>), grid, dim3(256), 0, st, j); break;
    case 256: ZASR_LAUNCH((joiner_split_kernel<4, NP, FMT>), grid, dim3(256), 0, st, j); break;
    case 512: ZASR_LAUNCH((joiner_split_kernel<8, NP, FMT>), grid, dim3(256), 0, st, j); break;
    default: throw std::runtime_error("joiner dim must be 64, 128, 256 or 512");
  }
}

// --------------------------------------------------------------------------------------
// speculative-greedy / beam joiner on fragment-packed J / W (kernels.h JoinerPackedArgs).
// Register-staged: no LDS.  Each wave streams its own J row tile and W column group (1 KB
// coalesced fragment loads, 8 fragments of each in flight ahead of the MFMAs) -- twice the L2
// reads of an LDS-shared tile, but a block needs no LDS and few VGPRs, so under the batch
// pipeline it co-resides with the next batch's encoder GEMM blocks instead of waiting for whole
// CUs to drain.
template <int QK>
__global__ __launch_bounds__(256) void joiner_reg_kernel(JoinerPackedArgs j) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * 64;
  if (tile_done(j.live_t, j.live_len, j.live_f, m0, j.M) &&
      (m0 + 32 >= j.M || tile_done(j.live_t, j.live_len, j.live_f, m0 + 32, j.M)))
    return;  // block-uniform: every stream of these 64 rows has finished
  const int rt = wid >> 1, gc = wid & 1;
  const int row0 = m0 + 32 * rt;
  const int g = blockIdx.x * 2 + gc;
  if (row0 >= j.M || g * 32 >= j.V) return;
  const bf16x8* srcJ = reinterpret_cast<const bf16x8*>(j.Jp) + (long)(row0 >> 5) * QK * 64 + lane;
  const bf16x8* srcW = reinterpret_cast<const bf16x8*>(j.Wp) + (long)g * QK * 64 + lane;
  constexpr int CH = 8;
  constexpr int NCH = QK / CH;
  bf16x8 a[2][CH], b[2][CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    a[0][c] = srcJ[c * 64];
    b[0][c] = srcW[c * 64];
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int h = 0; h < NCH; ++h) {
    const int cur = h & 1;
    if (h + 1 < NCH) {
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        a[cur ^ 1][c] = srcJ[((h + 1) * CH + c) * 64];
        b[cur ^ 1][c] = srcW[((h + 1) * CH + c) * 64];
      }
    }
#pragma unroll
    for (int c = 0; c < CH; ++c)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cur][c], b[cur][c], acc, 0, 0, 0);
  }
  const int col = g * 32 + (lane & 31);
  if (col >= j.V) return;
  const float bb = j.bias[col];
  const int hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (row < j.M) j.out[(long)row * j.V + col] = acc[r] + bb;
  }
}

// Split-bf16 modes on packed pieces: the joiner_reg_kernel structure (no LDS: co-resides with
// the encoder blocks of the next batch), each k16 step loading the NP pieces of its J and W
// fragments (written / packed once: store_j4, Engine load) and issuing the NP (NP + 1) / 2
// piece products smallest first (mfma_split, the order of gemm_x3 / joiner_split_kernel).
// CH k16 steps of fragments in flight per register set.
template <int QK, int NP, int CH, int FMT = 0>
__global__ __launch_bounds__(256) void joiner_split_packed_kernel(JoinerPackedArgs j) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.y * 64;
  if (tile_done(j.live_t, j.live_len, j.live_f, m0, j.M) &&
      (m0 + 32 >= j.M || tile_done(j.live_t, j.live_len, j.live_f, m0 + 32, j.M)))
    return;  // block-uniform: every stream of these 64 rows has finished
  const int rt = wid >> 1, gc = wid & 1;
  const int row0 = m0 + 32 * rt;
  const int g = blockIdx.x * 2 + gc;
  if (row0 >= j.M || g * 32 >= j.V) return;
  const bf16x8* srcJ = reinterpret_cast<const bf16x8*>(j.Jp) + (long)(row0 >> 5) * QK * 64 + lane;
  const bf16x8* srcW = reinterpret_cast<const bf16x8*>(j.Wp) + (long)g * QK * 64 + lane;
  const long jp = j.j_plane / 8, wp = j.w_plane / 8;  // planes in bf16x8 units
  constexpr int NCH = QK / CH;
  bf16x8 a[2][CH][NP], b[2][CH][NP];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      a[0][c][t] = srcJ[t * jp + c * 64];
      b[0][c][t] = srcW[t * wp + c * 64];
    }
  f32x16 acc, accl;  // accl: the lo products (FMT 1, the f16x3 format)
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = accl[r] = 0.f;
  // the next set's loads go out as one group before this set's MFMAs (scheduling barriers:
  // left alone, the compiler streams one load per MFMA with ~4 in flight, latency-bound)
#pragma unroll
  for (int h = 0; h < NCH; ++h) {
    const int cur = h & 1;
    if (h + 1 < NCH) {
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int t = 0; t < NP; ++t) {
          a[cur ^ 1][c][t] = srcJ[t * jp + ((h + 1) * CH + c) * 64];
          b[cur ^ 1][c][t] = srcW[t * wp + ((h + 1) * CH + c) * 64];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if constexpr (FMT == 1) {
        const bf16x8 x[2] = {a[cur][c][0], a[cur][c][1]};
        const bf16x8 y[2] = {b[cur][c][0], b[cur][c][1]};
        mfma_h3(x, y, acc, accl);
      } else {
        acc = mfma_split<NP>(a[cur][c], b[cur][c], acc);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (FMT == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += accl[r] * kF16LoInv;
  }
  const int col = g * 32 + (lane & 31);
  if (col >= j.V) return;
  const float bb = j.bias[col];
  const int hh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
    if (row < j.M) j.out[(long)row * j.V + col] = acc[r] + bb;
  }
}

void launch_joiner_packed(const JoinerPackedArgs& j, hipStream_t st) {
  if (j.M <= 0) return;
  dim3 grid(cdiv(j.V, 64), cdiv(j.M, 64));
  if (j.pieces > 0) {
    ZASR_REQUIRE(j.pieces == 2 || j.pieces == 3 || j.pieces == kPiecesF16,
                 "packed split joiner: pieces must be 2, 3 or kPiecesF16");
    ZASR_REQUIRE(j.D == 256 || j.D == 512, "packed split joiner: joiner dim must be 256 or 512");
    const int qk = j.D / 16;
    if (j.pieces == kPiecesF16) {
      if (qk == 16) ZASR_LAUNCH((joiner_split_packed_kernel<16, 2, 4, 1>), grid, dim3(256), 0, st, j);
      else ZASR_LAUNCH((joiner_split_packed_kernel<32, 2, 4, 1>), grid, dim3(256), 0, st, j);
    } else if (j.pieces == 2) {
      if (qk == 16) ZASR_LAUNCH((joiner_split_packed_kernel<16, 2, 4>), grid, dim3(256), 0, st, j);
      else ZASR_LAUNCH((joiner_split_packed_kernel<32, 2, 4>), grid, dim3(256), 0, st, j);
    } else {
      if (qk == 16) ZASR_LAUNCH((joiner_split_packed_kernel<16, 3, 4>), grid, dim3(256), 0, st, j);
      else ZASR_LAUNCH((joiner_split_packed_kernel<32, 3, 4>), grid, dim3(256), 0, st, j);
    }
    return;
  }
  // (an LDS-shared variant, every operand by LDS-DMA, measured 12 % slower under the batch
  // pipeline: it needs whole CUs)
  switch (j.D) {
    case 256: ZASR_LAUNCH(joiner_reg_kernel<16>, grid, dim3(256), 0, st, j); break;
    case 512: ZASR_LAUNCH(joiner_reg_kernel<32>, grid, dim3(256), 0, st, j); break;
    default: throw std::runtime_error("packed joiner: joiner dim must be 256 or 512");
  }
}

// element offset of J[row][k] in the fragment-packed image (kernels.h JoinerPackedArgs)
__device__ __forceinline__ long packed_j_off(long row, int k, int D) {
  const long rt = row >> 5;
  const int r = (int)(row & 31), q = k >> 4, hh = (k >> 3) & 1, j = k & 7;
  return ((rt * (D >> 4) + q) * 64 + r + 32 * hh) * 8 + j;
}

__device__ __forceinline__ void store_j4(const DecTable& dt, long row, int k, float4 e, float4 d) {
  if (dt.j_packed && dt.j_pieces > 0) {
    // split-bf16 modes: the f32 J of the f32 path (tanhf), written once as bf16 pieces in
    // fragment order, so the joiner reads ready MFMA operands (no per-launch split)
    float r[4] = {tanhf(e.x + d.x), tanhf(e.y + d.y), tanhf(e.z + d.z), tanhf(e.w + d.w)};
    __bf16* base = reinterpret_cast<__bf16*>(dt.J) + packed_j_off(row, k, dt.D);
    if (dt.j_pieces == kPiecesF16) {  // fp16 hi, (x - hi) * 2^11 (gemm_dev.h split_h8)
      bf16x4 vh, vl;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const _Float16 hh = (_Float16)r[q];
        vh[q] = __builtin_bit_cast(__bf16, hh);
        vl[q] = __builtin_bit_cast(__bf16, (_Float16)((r[q] - (float)hh) * kF16Lo));
      }
      *reinterpret_cast<bf16x4*>(base) = vh;
      *reinterpret_cast<bf16x4*>(base + dt.j_plane) = vl;
      return;
    }
    for (int t = 0; t < dt.j_pieces; ++t) {
      bf16x4 v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        v[q] = (__bf16)r[q];
        r[q] -= (float)v[q];
      }
      *reinterpret_cast<bf16x4*>(base + t * dt.j_plane) = v;
    }
  } else if (dt.j_packed) {  // 4 consecutive k stay inside one 8-element fragment slot
    bf16x4 v;
    v[0] = (__bf16)fast_tanh(e.x + d.x);
    v[1] = (__bf16)fast_tanh(e.y + d.y);
    v[2] = (__bf16)fast_tanh(e.z + d.z);
    v[3] = (__bf16)fast_tanh(e.w + d.w);
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(dt.J) + packed_j_off(row, k, dt.D)) = v;
  } else if (dt.j_bf16) {
    bf16x4 v;
    v[0] = (__bf16)fast_tanh(e.x + d.x);
    v[1] = (__bf16)fast_tanh(e.y + d.y);
    v[2] = (__bf16)fast_tanh(e.z + d.z);
    v[3] = (__bf16)fast_tanh(e.w + d.w);
    *reinterpret_cast<bf16x4*>(reinterpret_cast<__bf16*>(dt.J) + row * dt.D + k) = v;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(dt.J) + row * dt.D + k) =
        make_float4(tanhf(e.x + d.x), tanhf(e.y + d.y), tanhf(e.z + d.z), tanhf(e.w + d.w));
  }
}

// f16x3 guard: *flag = 1 when any of the n floats is not finite (an activation beyond the
// fp16 range became inf in a split and spread); read back with the search results
__global__ void nonfinite_kernel(const float4* __restrict__ x, long n4, int* __restrict__ flag) {
  bool bad = false;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = x[i];
    bad |= !(__builtin_isfinite(v.x) && __builtin_isfinite(v.y) && __builtin_isfinite(v.z) &&
             __builtin_isfinite(v.w));
  }
  if (bad) *flag = 1;
}

void launch_nonfinite_check(const float* x, long n, int* flag, hipStream_t st) {
  ZASR_REQUIRE(n % 4 == 0, "nonfinite check: n must be a multiple of 4");
  ZASR_HIP_CHECK(hipMemsetAsync(flag, 0, sizeof(int), st));
  if (n <= 0) return;
  const long n4 = n / 4;
  const int blocks = (int)std::min<long>(cdivl(n4, 256), 2048);
  ZASR_LAUNCH(nonfinite_kernel, dim3(blocks), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(x), n4, flag);
}

// J of frame 0, slot 0 of stream s: context (0, 0) = table row 0
__global__ void table_init_kernel(DecTable dt, int S, int Hmax) {
  const int d4 = dt.D / 4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)S * d4) return;
  const int s = (int)(i / d4), c4 = (int)(i - (long)s * d4);
  if (dt.enc_len[s] <= 0) return;
  const float4 e = *reinterpret_cast<const float4*>(dt.enc + (long)dt.enc_off[s] * dt.D + 4 * c4);
  const float4 d = *reinterpret_cast<const float4*>(dt.table + 4 * c4);
  store_j4(dt, (long)s * Hmax, 4 * c4, e, d);
}

void launch_table_init(const DecTable& dt, int S, int Hmax, hipStream_t st) {
  if (S <= 0) return;
  ZASR_REQUIRE(dt.D % 4 == 0, "joiner dim must be a multiple of 4");
  const long n = (long)S * (dt.D / 4);
  ZASR_LAUNCH(table_init_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st, dt, S, Hmax);
}

// --------------------------------------------------------------------------------------
// One block of 8 waves per stream; hypothesis row h belongs to wave h % 8 (one row per wave
// up to beam 8).  Per row the wave
//   1. loads the row (float4 per lane, Q per lane) and reduces its statistics with DPP;
//   2. finds the row's top KB candidates: a threshold t = the smallest of KB disjoint lane
//      groups' maxima (every group holds an element >= t, so the row's top KB are >= t),
//      the elements >= t compacted into a per-wave LDS list by ballot, one per lane, keyed by
//      (candidate lp desc, flat index asc) -- the order this build gives the reference's
//      argpartition / argsort (core/asr_engine.py:1103-1106) -- and ranked by counting.  The
//      lp = ((x - max) - log S) + score_h is monotone in x, so an element below t can only
//      reach the list by an f32 rounding tie with the KB-th lp; when the KB-th lp equals lp(t)
//      (or more than 64 elements pass t) the row takes the exact slow path: elements popped
//      in (x desc, index asc) order until the KB-th and its lp ties;
//   3. decodes its KB best (token, hotword transition :1127-1131, sequence identity) into LDS
//      slots h * KB + rank, so the hotword table loads overlap the other rows.
// After one block barrier wave 0 ranks the n * KB slots, merges duplicates and writes the new
// hypotheses; then every wave writes the next frame's joiner input of its candidates.
#ifdef ZASR_SEARCH_STAMPS  // development: per-phase shader cycles of block 0, wave 0
__device__ unsigned long long g_ss_sum[12];
__device__ unsigned long long g_ss_n;
#define SS_STAMP(i) \
  if (ss_on) ss_t[i] = __builtin_amdgcn_s_memtime();
#else
#define SS_STAMP(i)
#endif
template <int KB, int Q, bool TABLE>
__global__ __launch_bounds__(512) void search_step_kernel(SearchState st, const float* logits,
                                                          int V, int Hmax, int beam, int t,
                                                          const int* enc_len, HotwordTables hw,
                                                          DecTable dt) {
  constexpr int NW = 8;
  constexpr int NKS = KB * KB;  // row h's list in slots h * KB + r (n <= beam <= KB rows)
  const int s = blockIdx.x;
  const int T_s = enc_len[s];
  if (t >= T_s) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int base = s * Hmax;
#ifdef ZASR_SEARCH_STAMPS
  const bool ss_on = s == 0 && tid == 0;
  unsigned long long ss_t[12];
#endif
  SS_STAMP(0)

  __shared__ float4 sStats[kMaxBeam];
  __shared__ unsigned long long cK[NKS], dHash[NKS];
  __shared__ double dScore[NKS];
  __shared__ float dVal[NKS];
  __shared__ int dHi[NKS], dTok[NKS], dLen[NKS], dY1[NKS], dY2[NKS], dHw[NKS];
  __shared__ float wX[NW][64];
  __shared__ int wI[NW][64];
  __shared__ int cSrc[kMaxBeam], cDup[kMaxBeam];
  __shared__ int sKK;
  __shared__ unsigned long long sFmask;

  const int V4 = V >> 2;
  const float4* rows4 = reinterpret_cast<const float4*>(logits + (long)base * V);
  // this wave's first row, issued before anything else (rows >= nh hold stale but valid data)
  float4 xa[Q];
  double ld_cur = 0.0;
  int lpf_cur = 0;
  if (wid < Hmax) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane + 64 * q;
      xa[q] = i < V4 ? rows4[(long)wid * V4 + i] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
    ld_cur = st.lp[base + wid];
    lpf_cur = st.lpf[base + wid];
  }
  // every wave holds the hypothesis records in lanes < Hmax (slots >= nh are stale but valid
  // memory and never selected)
  double pLp = 0.0;
  unsigned long long pHash = 0ull;
  int pLen = 0, pY1 = 0, pY2 = 0, pHw = 0, pNode = 0;
  if (lane < Hmax) {
    pLp = st.lp[base + lane];
    pHash = st.hash[base + lane];
    pLen = st.len[base + lane];
    pY1 = st.y1[base + lane];
    pY2 = st.y2[base + lane];
    pHw = st.hw[base + lane];
    pNode = st.node[base + lane];
  }
  const int node_base = st.node_count[s];
  const int n = st.nh[s];
  const bool use_hw = hw.num_states > 0;
  // the next frame's encoder row (every wave writes J rows of candidates in step 4)
  float4 ev[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  const bool next = t + 1 < T_s;
  if constexpr (TABLE) {
    if (next) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c4 = lane + 64 * j;
        if (c4 < dt.D / 4)
          ev[j] = *reinterpret_cast<const float4*>(dt.enc + (long)(dt.enc_off[s] + t + 1) * dt.D + 4 * c4);
      }
    }
  }

  // ---- 1 + 2. per row: statistics (:1096-1098, :1159-1181) and the row's top candidates ----
  //   max / second max; S = sum e, E1 = sum e d, E3 = sum exp(d / 3) (d = x - max):
  //   entropy = log S - E1 / S, sum p^(1/3) = S^(-1/3) E3, top1 = 1 / S, top2 = e^(m2-m1) / S
  //   candidate lp = ((x - max) - log S) + score_h (f32 add of the Python-float score, or the
  //   f64 add of an np.float64 score, :1099-1100)
  for (int h = wid; h < n; h += NW) {
    if (h != wid) {  // beam > 8: a second row per wave
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const int i = lane + 64 * q;
        xa[q] = i < V4 ? rows4[(long)h * V4 + i] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      }
      ld_cur = st.lp[base + h];
      lpf_cur = st.lpf[base + h];
    }
    float m1 = -INFINITY, m2 = -INFINITY;
    auto upd = [&](float x) {  // branch-free (a branchy form put m1/m2 in scratch)
      m2 = fmaxf(m2, fminf(m1, x));
      m1 = fmaxf(m1, x);
    };
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      upd(xa[q].x);
      upd(xa[q].y);
      upd(xa[q].z);
      upd(xa[q].w);
    }
    // candidate threshold: lane groups (DPP): KB >= 16: the 16 quads; KB = 8: overlapping
    // quad pairs (q, q - 1), of which the 8 pairs (2i, 2i + 1) are disjoint, so the minimum
    // over all of them is still a bound; KB <= 4: the four 16-lane rows
    float thr_x = fmaxf(m1, dpp_f<kDppQuad1>(m1));
    thr_x = fmaxf(thr_x, dpp_f<kDppQuad2>(thr_x));
    if constexpr (KB <= 8) thr_x = fmaxf(thr_x, dpp_f<kDppRor4>(thr_x));
    if constexpr (KB <= 4) thr_x = fmaxf(thr_x, dpp_f<kDppRor8>(thr_x));
    thr_x = wave_min_dpp(thr_x);
    wave_max2_dpp(m1, m2);
    SS_STAMP(1)
    float se = 0.f, e1 = 0.f, e3 = 0.f;
    auto acc = [&](float x) {
      const float d = x - m1;  // -inf past V -> e = 0
      const float e = __expf(d);
      se += e;
      e1 = (e > 0.f) ? fmaf(e, d, e1) : e1;
      e3 += __expf(d * (1.0f / 3.0f));
    };
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      acc(xa[q].x);
      acc(xa[q].y);
      acc(xa[q].z);
      acc(xa[q].w);
    }
    se = wave_sum_dpp(se);
    e1 = wave_sum_dpp(e1);
    e3 = wave_sum_dpp(e3);
    const float ls = logf(se);
    if (lane == 0)
      sStats[h] = make_float4(ls - e1 / se, e3 * exp2f(-log2f(se) * (1.0f / 3.0f)), 1.0f / se,
                              __expf(m2 - m1) / se);
    SS_STAMP(2)
    const double ld = ld_cur;
    const bool f64 = lpf_cur != 0;
    const float lf = (float)ld;
    auto score = [&](float x) {
      const float lpv = (x - m1) - ls;
      return f64 ? (float)((double)lpv + ld) : lpv + lf;
    };
    // 2a. elements >= thr_x into the wave's list (order: q, component, lane)
    int total = 0;
    auto push = [&](float x, int col) {
      const bool p = x >= thr_x;
      const unsigned long long m = __ballot(p);
      if (m) {
        const int pos = total + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        if (p && pos < 64) {
          wX[wid][pos] = x;
          wI[wid][pos] = col;
        }
        total += __popcll(m);
      }
    };
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int c0 = 4 * (lane + 64 * q);
      push(xa[q].x, c0);
      push(xa[q].y, c0 + 1);
      push(xa[q].z, c0 + 2);
      push(xa[q].w, c0 + 3);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // 2b. keys and ranks within the row
    unsigned long long key = 0ull;
    float val = -INFINITY;
    int ncand = total;
    bool fast = total <= 64;
    // the hotword class of this lane's candidate token, fetched now so that the dependent
    // transition loads of step 2c are the only hotword round trip left behind the ranking
    int pcls = -1;
    if (fast) {
      if (lane < total) {
        const int col = wI[wid][lane];
        val = score(wX[wid][lane]);
        key = make_key(val, h * V + col);
#ifndef ZASR_NO_CLS_PREFETCH  // (A/B builds: tools/ab_variant.sh)
        if (use_hw) pcls = hw.tok2cls[col];
#endif
      }
    }
    int rank = 64;
    auto rank_keys = [&]() {
      rank = 0;
      for (int c = 0; c < ncand; ++c) rank += lane_u64(key, c) > key ? 1 : 0;
      if (lane >= ncand) rank = 64;
    };
    if (fast) {
      rank_keys();
      const unsigned long long kth = __ballot(rank == KB - 1);
      // exact unless an element below the threshold can tie the KB-th lp
      fast = kth != 0ull && lane_f(val, __ffsll((long long)kth) - 1) != score(thr_x);
    }
    if (!fast) {
      // slow path: pop in (x desc, index asc) order -- per lane the head and second of its
      // elements, the popped lane promoting its second or rescanning what follows -- until
      // the KB-th and every further element with an equal lp
      float hv = -INFINITY, sv = -INFINITY;
      int hj = -1, sj = -1;
      auto take = [&](float x, int j) {  // strict >: the earlier of equal values ranks first
        const bool gh = x > hv, gs = x > sv;
        sv = gh ? hv : (gs ? x : sv);
        sj = gh ? hj : (gs ? j : sj);
        hv = gh ? x : hv;
        hj = gh ? j : hj;
      };
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        take(xa[q].x, 4 * q);
        take(xa[q].y, 4 * q + 1);
        take(xa[q].z, 4 * q + 2);
        take(xa[q].w, 4 * q + 3);
      }
      bool sv_ok = true;
      float s_kb = 0.f;
      int got = 0;  // wave-uniform
      key = 0ull;
      for (;;) {
        const float g = wave_max_dpp(hv);
        if (g == -INFINITY) break;  // row exhausted
        const unsigned long long tied = __ballot(hv == g);
        const int myidx = 4 * (lane + 64 * (hj >> 2)) + (hj & 3);
        int owner;
        if (__popcll(tied) == 1) {
          owner = __ffsll((long long)tied) - 1;
        } else {  // equal heads in several lanes: the smallest column first
          const int mi = wave_min_i_dpp(hv == g ? myidx : 0x7fffffff);
          owner = __ffsll((long long)__ballot(hv == g && myidx == mi)) - 1;
        }
        const int gidx = __builtin_amdgcn_readlane(myidx, owner);
        const float v = score(g);
        if (got >= KB && v != s_kb) break;  // past the KB-th and its lp ties
        if (got >= 64) break;               // > 56 equal f32 lps: never seen
        if (got == KB - 1) s_kb = v;
        if (lane == got) key = make_key(v, h * V + gidx);
        ++got;
        if (lane == owner) {  // pop: promote the second, or rescan what follows the popped one
          const float pv = hv;
          const int pj = hj;
          if (sv_ok) {
            hv = sv;
            hj = sj;
            sv_ok = false;
          } else {
            hv = sv = -INFINITY;
            hj = sj = -1;
            auto after = [&](float x, int j) {
              if (x < pv || (x == pv && j > pj)) take(x, j);
            };
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              after(xa[q].x, 4 * q);
              after(xa[q].y, 4 * q + 1);
              after(xa[q].z, 4 * q + 2);
              after(xa[q].w, 4 * q + 3);
            }
            sv_ok = true;
          }
        }
      }
      ncand = got;
      rank_keys();
    }
    SS_STAMP(3)
    // 2c. the row's KB best -> slots h * KB + rank, decoded (:1116-1131): blank keeps the
    //     sequence, non-blank appends and steps the hotword graph (blank and UNK skip it,
    //     :1129); every lane < KB writes its slot (empty: key 0)
    {
      const unsigned long long phash = lane_u64(pHash, h);
      const int plen = __builtin_amdgcn_readlane(pLen, h);
      const int py1 = __builtin_amdgcn_readlane(pY1, h);
      const int py2 = __builtin_amdgcn_readlane(pY2, h);
      const int phw = __builtin_amdgcn_readlane(pHw, h);
      if (lane < KB) cK[h * KB + lane] = 0ull;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      if (rank < KB) {
        const int slot = h * KB + rank;
        const int tok = key_idx(key) - h * V;
        double sc = (double)key_val(key);
        int nhw = phw, klen, ny1, ny2;
        unsigned long long hk;
        if (tok == 0) {
          hk = phash;
          klen = plen;
          ny1 = py1;
          ny2 = py2;
        } else {
          if (use_hw && tok != 2) {
#ifndef ZASR_NO_CLS_PREFETCH
            // the fast path kept each candidate in the lane that fetched its class
            const int cls = fast ? pcls : hw.tok2cls[tok];
#else
            const int cls = hw.tok2cls[tok];
#endif
            if (cls < 0) {
              sc += -hw.node_score[nhw];
              nhw = 0;
            } else {
              const long e = (long)nhw * hw.num_cls + cls;
              sc += hw.delta[e];
              nhw = hw.next[e];
            }
          }
          hk = hash_push(phash, tok);
          klen = plen + 1;
          ny2 = py1;
          ny1 = tok;
        }
        cK[slot] = key;
        dVal[slot] = key_val(key);
        dHi[slot] = h;
        dTok[slot] = tok;
        dScore[slot] = sc;
        dHw[slot] = nhw;
        dHash[slot] = hk;
        dLen[slot] = klen;
        dY1[slot] = ny1;
        dY2[slot] = ny2;
      }
    }
  }
  SS_STAMP(4)
  __syncthreads();
  SS_STAMP(5)
  // ---- 3. expansion (:1110-1138): ranking and duplicate merge in wave 0 ----
  const int total_c = n * V;
  const int k = beam < total_c ? beam : total_c;
  const int nk = n * KB;
  if (wid == 0) {
    // 3a. global rank of each slot key (keys are distinct): the k best, best first
    int nz = 0;
#pragma unroll
    for (int r0 = 0; r0 < NKS; r0 += 64) {
      const int c = r0 + lane;
      const unsigned long long key = c < nk ? cK[c] : 0ull;
      int rank = 0;
      for (int j = 0; j < nk; ++j) rank += cK[j] > key ? 1 : 0;
      if (key != 0ull && rank < k) cSrc[rank] = c;
      nz += __popcll(__ballot(key != 0ull));
    }
    const int kk = k < nz ? k : nz;
    if (lane == 0) sKK = kk;
    SS_STAMP(6)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // 3b. duplicates of the full sequence merge into their first occurrence, in candidate
    //     order, with an f64 log-add (:1133-1138)
    const bool lv = lane < kk;
    const int src = lv ? cSrc[lane] : 0;
    const unsigned long long key = lv ? dHash[src] : 0ull;
    const int klen = lv ? dLen[src] : 0;
    int dup = -1;
    if (lv) {
      for (int c = 0; c < lane; ++c) {
        const int o = cSrc[c];
        if (dLen[o] == klen && dHash[o] == key) {
          dup = c;
          break;
        }
      }
      cDup[lane] = dup;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const bool first = lv && dup < 0;
    const int tok = lv ? dTok[src] : 0;
    const int hi = lv ? dHi[src] : 0;
    const double plp = shfl_f64(pLp, hi);
    const int pnode = __shfl(pNode, hi);
    const unsigned long long fmask = __ballot(first);
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int slot = __popcll(fmask & below);
    const bool emit = first && tok != 0;
    const unsigned long long emask = __ballot(emit);
    if (first) {
      double lp = dScore[src];
      int f64 = 0;
      for (int c = lane + 1; c < kk; ++c)
        if (cDup[c] == lane) lp = log_add(lp, f64, dScore[cSrc[c]], 0, &f64);
      int nnode = pnode;
      if (emit) {
        const int nid = node_base + __popcll(emask & below);
        const long gi = (long)s * st.node_cap + nid;
        st.node_tok[gi] = tok;
        st.node_frame[gi] = t;
        st.node_parent[gi] = pnode;
        st.node_lp[gi] = (double)dVal[src] - plp;
        st.node_stats[gi] = sStats[hi];
        nnode = nid;
      }
      const int o = base + slot;
      st.lp[o] = lp;
      st.lpf[o] = f64;
      st.hash[o] = key;
      st.len[o] = klen;
      st.y1[o] = dY1[src];
      st.y2[o] = dY2[src];
      st.hw[o] = dHw[src];
      st.node[o] = nnode;
    }
    if (lane == 0) {
      st.nh[s] = __popcll(fmask);
      st.node_count[s] = node_base + __popcll(emask);
      sFmask = fmask;
    }
    SS_STAMP(7)
  }
  // ---- 4. the next frame's joiner input J[slot] = tanh(enc[s, t + 1] + table[context]),
  //         candidate c by wave c % 8 ----
  if constexpr (TABLE) {
    if (next) {
      __syncthreads();  // sFmask, sKK, cSrc
      SS_STAMP(8)
      const unsigned long long fm = sFmask;
      const int kk_all = sKK;
      for (int cc = wid; cc < kk_all; cc += NW) {
        if (!((fm >> cc) & 1ull)) continue;
        const int src = cSrc[cc];
        const float* row = dt.table + ((long)dY2[src] * dt.V + dY1[src]) * dt.D;
        const int sl = __popcll(fm & ((1ull << cc) - 1ull));
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c4 = lane + 64 * j;
          if (c4 < dt.D / 4)
            store_j4(dt, base + sl, 4 * c4, ev[j], *reinterpret_cast<const float4*>(row + 4 * c4));
        }
      }
    }
  }
#ifdef ZASR_SEARCH_STAMPS
  if (ss_on) {
    ss_t[9] = __builtin_amdgcn_s_memtime();
    if (next) {
      for (int q = 1; q < 10; ++q) atomicAdd(&g_ss_sum[q], ss_t[q] - ss_t[q - 1]);
      atomicAdd(&g_ss_n, 1ull);
    } else {
      const unsigned long long n = g_ss_n > 0 ? g_ss_n : 1;
      printf("[search stamps] frames %llu mean cycles: max %llu stats %llu topk %llu decode %llu "
             "barrier %llu rank %llu tail %llu barrier2 %llu J %llu\n", g_ss_n, g_ss_sum[1] / n,
             g_ss_sum[2] / n, g_ss_sum[3] / n, g_ss_sum[4] / n, g_ss_sum[5] / n, g_ss_sum[6] / n,
             g_ss_sum[7] / n, g_ss_sum[8] / n, g_ss_sum[9] / n);
      for (int q = 0; q < 12; ++q) g_ss_sum[q] = 0;
      g_ss_n = 0;
    }
  }
#endif
}

void launch_search_step(const SearchState& s, const float* logits, int V, int S, int Hmax,
                        int beam, int t, const int* enc_len, const HotwordTables& hw,
                        const DecTable* dt, hipStream_t st) {
  if (S <= 0) return;
  ZASR_REQUIRE(beam >= 1 && beam <= kMaxBeam && beam <= Hmax, "beam out of range");
  ZASR_REQUIRE(V % 4 == 0 && V <= 4096, "vocabulary size must be a multiple of 4, <= 4096");
  ZASR_REQUIRE(!dt || (dt->D % 4 == 0 && dt->D <= 512), "joiner dim must be a multiple of 4, <= 512");
  dim3 grid(S), block(512);
  DecTable d{};
  if (dt) d = *dt;
#define ZASR_STEP3(KBV, QV)                                                                 \
  do {                                                                                      \
    if (dt)                                                                                 \
      ZASR_LAUNCH((search_step_kernel<KBV, QV, true>), grid, block, 0, st, s, logits, \
                         V, Hmax, beam, t, enc_len, hw, d);                                 \
    else                                                                                    \
      ZASR_LAUNCH((search_step_kernel<KBV, QV, false>), grid, block, 0, st, s,        \
                         logits, V, Hmax, beam, t, enc_len, hw, d);                         \
  } while (0)
#define ZASR_STEP(KBV)             \
  do {                             \
    if (V <= 512)                  \
      ZASR_STEP3(KBV, 2);          \
    else if (V <= 2048)            \
      ZASR_STEP3(KBV, 8);          \
    else                           \
      ZASR_STEP3(KBV, 16);         \
  } while (0)
  if (beam == 1) {
    ZASR_STEP(1);
  } else if (beam <= 4) {
    ZASR_STEP(4);
  } else if (beam <= 8) {
    ZASR_STEP(8);
  } else {
    ZASR_STEP(16);
  }
#undef ZASR_STEP
#undef ZASR_STEP3
}

// --------------------------------------------------------------------------------------
// speculative greedy (kernels.h).  J of the first window: frames 0 .. F-1, context (0, 0).
// --------------------------------------------------------------------------------------
__global__ void greedy_spec_init_kernel(DecTable dt, int S, int F, int* t_cur, int* active) {
  const int d4 = dt.D / 4;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2) active[i] = 0;
  if (i >= (long)S * F * d4) return;
  const int c4 = (int)(i % d4);
  const long sf = i / d4;
  const int s = (int)(sf / F), f = (int)(sf - (long)s * F);
  if (f == 0 && c4 == 0) t_cur[s] = 0;
  if (f >= dt.enc_len[s]) return;
  const float4 e = *reinterpret_cast<const float4*>(dt.enc + (long)(dt.enc_off[s] + f) * dt.D + 4 * c4);
  const float4 d = *reinterpret_cast<const float4*>(dt.table + 4 * c4);
  store_j4(dt, sf, 4 * c4, e, d);
}

void launch_greedy_spec_init(const DecTable& dt, int S, int F, int* t_cur, int* active,
                             hipStream_t st) {
  if (S <= 0) return;
  ZASR_REQUIRE(dt.D % 4 == 0, "joiner dim must be a multiple of 4");
  const long n = std::max<long>((long)S * F * (dt.D / 4), 2);
  ZASR_LAUNCH(greedy_spec_init_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st,
                     dt, S, F, t_cur, active);
}

// One block per stream, wave w owns window rows w, w + 4, ... (register resident).
//   A. per row: max, second max, log S (S = sum e), and d0 = fl(x_blank - max); the
//      encoder rows of every frame the next window can start at (t0 + 1 .. t0 + 2F - 1) and
//      the current context's table row are staged in LDS meanwhile
//   B. lf_f = the score before frame f if frames 0 .. f-1 were all blank: the reference's
//      f32 recurrence lp <- fl(fl(d0 - log S) + fl(lp)) (one thread)
//   C. per row, the top-1 of search_step_kernel's candidate order: the value
//      fl(fl(fl(x - max) - log S) + lf_f) is monotone in x, so the top value is that of x =
//      max and the winner is the smallest index reaching it (a float compare per element)
//   D. the first non-blank row is the emission: its owning wave adds the entropy terms of
//      that row and writes node + state (hotword transition :1127-1131); all waves write the
//      next window's J rows from the staged encoder rows and the (new) context's table row
template <int F, int Q>
__global__ __launch_bounds__(256) void greedy_spec_kernel(SearchState st, const float* logits,
                                                          int V, int* t_cur, const int* enc_len,
                                                          HotwordTables hw, DecTable dt,
                                                          int* active, int parity) {
  constexpr int RPW = F / 4;  // rows per wave
  constexpr int DMAX = 512;
  const int s = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (s == 0 && tid == 0) active[parity ^ 1] = 0;  // the next super-step's counter
  const int T_s = enc_len[s];
  const int t0 = t_cur[s];
  if (t0 >= T_s) return;
  const int nf = T_s - t0 < F ? T_s - t0 : F;
  const int V4 = V >> 2;
  const int D = dt.D, d4 = D >> 2;
  __shared__ float sLs[F], sD0[F], sLf[F];
  __shared__ double sLp[F + 1];
  __shared__ int sTok[F];
  __shared__ float4 sEnc[(2 * F - 1) * (DMAX / 4)];
  __shared__ float4 sTab[DMAX / 4];
  const int base = s;  // Hmax = 1 at beam 1
  const int y1 = st.y1[base], y2 = st.y2[base];

  // ---- A. rows in registers; encoder rows t0 + 1 .. and the context row into LDS ----
  const float4* rows4 = reinterpret_cast<const float4*>(logits + (long)s * F * V);
  float4 x[RPW][Q];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int f = wid + 4 * r;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane + 64 * q;
      x[r][q] = (f < nf && i < V4) ? rows4[(long)f * V4 + i]
                                   : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
  }
  {
    const float4* enc4 = reinterpret_cast<const float4*>(dt.enc + (long)dt.enc_off[s] * D);
    const float4* tab4 = reinterpret_cast<const float4*>(dt.table + ((long)y2 * dt.V + y1) * D);
    constexpr int NE = (2 * F - 1) * (DMAX / 4);
    constexpr int IT = (NE + 255) / 256;
    float4 ev[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int e = tid + 256 * k;
      const int fr = e / d4, c4 = e - fr * d4;
      int t = t0 + 1 + fr;
      t = t < T_s ? t : T_s - 1;
      ev[k] = (fr < 2 * F - 1) ? enc4[(long)t * d4 + c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const float4 tv = tid < d4 ? tab4[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < IT; ++k) {
      const int e = tid + 256 * k;
      if (e < (2 * F - 1) * d4) sEnc[e] = ev[k];
    }
    if (tid < d4) sTab[tid] = tv;
  }
  float m1r[RPW], m2r[RPW], lsr[RPW], ser[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int f = wid + 4 * r;
    float m1 = -INFINITY, m2 = -INFINITY;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 v = x[r][q];
      m2 = fmaxf(m2, fminf(m1, v.x)); m1 = fmaxf(m1, v.x);
      m2 = fmaxf(m2, fminf(m1, v.y)); m1 = fmaxf(m1, v.y);
      m2 = fmaxf(m2, fminf(m1, v.z)); m1 = fmaxf(m1, v.z);
      m2 = fmaxf(m2, fminf(m1, v.w)); m1 = fmaxf(m1, v.w);
    }
    wave_max2_dpp(m1, m2);
    float se = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      se += __expf(x[r][q].x - m1);
      se += __expf(x[r][q].y - m1);
      se += __expf(x[r][q].z - m1);
      se += __expf(x[r][q].w - m1);
    }
    se = wave_sum_dpp(se);
    const float ls = logf(se);
    m1r[r] = m1;
    m2r[r] = m2;
    lsr[r] = ls;
    ser[r] = se;
    if (lane == 0 && f < nf) {
      sLs[f] = ls;
      sD0[f] = x[r][0].x - m1;  // blank = token 0 = lane 0's first element
    }
  }
  __syncthreads();
  // ---- B. scores before each frame under the all-blank hypothesis (f32 adds) ----
  if (tid == 0) {
    double lp = st.lp[base];
    sLp[0] = lp;
    for (int f = 0; f < nf; ++f) {
      const float lf = (float)lp;
      sLf[f] = lf;
      lp = (double)((sD0[f] - sLs[f]) + lf);
      sLp[f + 1] = lp;
    }
  }
  __syncthreads();
  // ---- C. top-1 token per row ----
  float4 pre[RPW][2];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int f = wid + 4 * r;
    if (f >= nf) continue;  // wave-uniform
    const float lf = sLf[f], m1 = m1r[r], ls = lsr[r];
    const float vmax = (0.f - ls) + lf;
    int bq = 0x7fffffff;
#pragma unroll
    for (int q = Q - 1; q >= 0; --q) {
      const int i = 4 * (lane + 64 * q);
      const float4 v = x[r][q];
      const int c = (((v.x - m1) - ls) + lf == vmax) ? i
                  : (((v.y - m1) - ls) + lf == vmax) ? i + 1
                  : (((v.z - m1) - ls) + lf == vmax) ? i + 2
                  : (((v.w - m1) - ls) + lf == vmax) ? i + 3 : 0x7fffffff;
      bq = c < bq ? c : bq;
    }
    // smallest index reaching the top value; a row with no match (non-finite logits, which
    // the encoder-output guard reports after the decode) reads as blank so that no index
    // derived from it leaves the vocabulary
    const int bm = wave_min_i_dpp(bq);
    const int best = bm < V ? bm : 0;
    if (lane == 0) sTok[f] = best;
    // a non-blank top-1 may be the window's emission: fetch the decoder-table row of the
    // context it would create now, under the block-wide decision below
    if (best != 0) {
      const float4* nrow = reinterpret_cast<const float4*>(dt.table + ((long)y1 * dt.V + best) * D);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c4 = lane + 64 * j;
        pre[r][j] = nrow[c4 < d4 ? c4 : d4 - 1];
      }
    }
  }
  __syncthreads();
  // ---- D. the first emission of the window ----
  int fe = -1;
  for (int f = 0; f < nf; ++f)
    if (sTok[f] != 0) {
      fe = f;
      break;
    }
  const int t_new = t0 + (fe >= 0 ? fe + 1 : nf);
  if (fe >= 0) {
    const int tok = sTok[fe];
    if ((fe & 3) == wid) {
      // owner wave: the entropy terms of row fe (search_step_kernel's statistics)
      // row r = fe >> 2 of this wave, chosen by selects (a dynamic register-array index
      // would put the arrays in scratch)
      const int r = fe >> 2;
      float m1 = m1r[0], m2 = m2r[0], se = ser[0], ls = lsr[0];
#pragma unroll
      for (int rr = 1; rr < RPW; ++rr) {
        m1 = rr == r ? m1r[rr] : m1;
        m2 = rr == r ? m2r[rr] : m2;
        se = rr == r ? ser[rr] : se;
        ls = rr == r ? lsr[rr] : ls;
      }
      float e1 = 0.f, e3 = 0.f;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        float4 v = x[0][q];
#pragma unroll
        for (int rr = 1; rr < RPW; ++rr) v = rr == r ? x[rr][q] : v;
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float d = vv[c] - m1;
          const float e = __expf(d);
          e1 = (e > 0.f) ? fmaf(e, d, e1) : e1;
          e3 += __expf(d * (1.0f / 3.0f));
        }
      }
      e1 = wave_sum_dpp(e1);
      e3 = wave_sum_dpp(e3);
      if (lane == 0) {
        const float val = (0.f - ls) + sLf[fe];
        double score = (double)val;
        int nhw = st.hw[base];
        if (hw.num_states > 0 && tok != 2) {
          const int cls = hw.tok2cls[tok];
          if (cls < 0) {
            score += -hw.node_score[nhw];
            nhw = 0;
          } else {
            const long e = (long)nhw * hw.num_cls + cls;
            score += hw.delta[e];
            nhw = hw.next[e];
          }
        }
        const int nid = st.node_count[s];
        const long gi = (long)s * st.node_cap + nid;
        st.node_tok[gi] = tok;
        st.node_frame[gi] = t0 + fe;
        st.node_parent[gi] = st.node[base];
        st.node_lp[gi] = (double)val - sLp[fe];
        st.node_stats[gi] = make_float4(ls - e1 / se, e3 * exp2f(-log2f(se) * (1.0f / 3.0f)),
                                        1.0f / se, __expf(m2 - m1) / se);
        st.node_count[s] = nid + 1;
        st.lp[base] = score;
        st.lpf[base] = 0;
        st.hash[base] = hash_push(st.hash[base], tok);
        st.len[base] = st.len[base] + 1;
        st.y2[base] = y1;
        st.y1[base] = tok;
        st.hw[base] = nhw;
        st.node[base] = nid;
      }
    }
  } else if (tid == 0) {
    st.lp[base] = sLp[nf];
    st.lpf[base] = 0;
  }
  if (tid == 0) {
    t_cur[s] = t_new;
    if (t_new < T_s) atomicAdd(&active[parity], 1);
  }
  // ---- the next window's joiner input: J[s][f] = tanh(enc[t_new + f] + table[ny2, ny1]) ----
  if (t_new >= T_s) return;
  const int nf2 = T_s - t_new < F ? T_s - t_new : F;
  if (fe >= 0 && (fe & 3) == wid) {
    // the emitting row's wave holds the new context's table row (prefetched in C)
    const int r = fe >> 2;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float4 v = pre[0][j];
#pragma unroll
      for (int rr = 1; rr < RPW; ++rr) v = rr == r ? pre[rr][j] : v;
      const int c4 = lane + 64 * j;
      if (c4 < d4) sTab[c4] = v;
    }
  }
  __syncthreads();
  const int fo = t_new - t0 - 1;  // staged row of frame t_new
  for (int e = tid; e < nf2 * d4; e += 256) {
    const int f = e / d4, c4 = e - f * d4;
    store_j4(dt, (long)s * F + f, 4 * c4, sEnc[(fo + f) * d4 + c4], sTab[c4]);
  }
}

void launch_greedy_spec(const SearchState& s, const float* logits, int V, int S, int F,
                        int* t_cur, const int* enc_len, const HotwordTables& hw,
                        const DecTable& dt, int* active, int parity, hipStream_t st) {
  if (S <= 0) return;
  ZASR_REQUIRE(V % 4 == 0 && V <= 4096, "vocabulary size must be a multiple of 4, <= 4096");
  ZASR_REQUIRE(dt.D % 4 == 0 && dt.D <= 512, "joiner dim must be a multiple of 4, <= 512");
#define ZASR_GS(FV, QV)                                                                      \
  ZASR_LAUNCH((greedy_spec_kernel<FV, QV>), dim3(S), dim3(256), 0, st, s, logits, V, \
                     t_cur, enc_len, hw, dt, active, parity)
  if (F == 4) {
    if (V <= 512) ZASR_GS(4, 2); else if (V <= 2048) ZASR_GS(4, 8); else ZASR_GS(4, 16);
  } else if (F == 8) {
    if (V <= 512) ZASR_GS(8, 2); else if (V <= 2048) ZASR_GS(8, 8); else ZASR_GS(8, 16);
  } else {
    throw std::runtime_error("greedy_spec: window must be 4 or 8 frames");
  }
#undef ZASR_GS
}

// --------------------------------------------------------------------------------------
// speculative greedy in ONE launch per super-step (kernels.h GreedyFusedArgs).
//
// Block (x, rt) = 8 waves over the joiner rows of row tile rt (32 rows = streams 8 rt ..
// 8 rt + 7, frames t_cur .. t_cur + 3) and the 256 vocabulary columns 256 x .. : wave w
// computes the 32 x 32 tile of column group 8 x + w over all of D with exactly the MFMA
// sequence of joiner_reg_kernel (bf16) / joiner_split_packed_kernel (f16x3), so the logits are
// those of the two-launch path bit for bit.  The logits leave by write-through (sc1) stores;
// after every wave's stores have completed, lane 0 adds one to the tile's arrival counter
// (agent scope) and the block that draws the last ticket runs the tile's greedy step, the
// logits read back by sc1 loads (MI355X_MICROARCH.md, inter-workgroup hand-off: sc1 stores +
// one agent-scope counter + sc1 loads, no fence).  No block waits for another, so the grid
// has no residency requirement.
//
// The greedy step of one stream is one wave (greedy_spec_kernel's four waves' work, the same
// operations in the same order per row): row statistics, the all-blank score recurrence, the
// top-1 of every window row, the first emission (node, state, hotword transition) and the
// next window's joiner input from the new context's table row.
namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t srch_rsrc(const void* p, long bytes) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)p);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long)p >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long)hi << 32) | lo), 0, n, 0x00020000);
}
constexpr int kCpolSc1 = 16;  // buffer cache-policy bit of sc1 (write-through / L1 bypass)
}  // namespace

template <int QK, int FMT, int Q>
__global__ __launch_bounds__(512) void joiner_greedy_kernel(GreedyFusedArgs a) {
  constexpr int F = 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rt = blockIdx.y, nct = gridDim.x;
  const JoinerPackedArgs& j = a.j;
  if (blockIdx.x == 0 && rt == 0 && tid == 0) a.active[a.parity ^ 1] = 0;  // the next step's count
  const int m0 = rt * 32;
  if (tile_done(a.t_cur, a.enc_len, F, m0, j.M)) return;  // block-uniform: all 8 streams done
  const __amdgpu_buffer_rsrc_t rso = srch_rsrc(j.out, (long)j.M * a.ldo * 4);

  // ---- joiner: wave w, column group g (32 columns), all 32 rows ----
  const int g = blockIdx.x * 8 + wid;
  if (g * 32 < j.V) {
    const bf16x8* srcJ = reinterpret_cast<const bf16x8*>(j.Jp) + (long)rt * QK * 64 + lane;
    const bf16x8* srcW = reinterpret_cast<const bf16x8*>(j.Wp) + (long)g * QK * 64 + lane;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    if constexpr (FMT == 0) {  // bf16: joiner_reg_kernel's loop
      constexpr int CH = 8, NCH = QK / CH;
      bf16x8 aa[2][CH], bb[2][CH];
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        aa[0][c] = srcJ[c * 64];
        bb[0][c] = srcW[c * 64];
      }
#pragma unroll
      for (int h = 0; h < NCH; ++h) {
        const int cur = h & 1;
        if (h + 1 < NCH) {
#pragma unroll
          for (int c = 0; c < CH; ++c) {
            aa[cur ^ 1][c] = srcJ[((h + 1) * CH + c) * 64];
            bb[cur ^ 1][c] = srcW[((h + 1) * CH + c) * 64];
          }
        }
#pragma unroll
        for (int c = 0; c < CH; ++c)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(aa[cur][c], bb[cur][c], acc, 0, 0, 0);
      }
    } else {  // f16x3: joiner_split_packed_kernel<QK, 2, 4, 1>'s loop
      constexpr int CH = 4, NCH = QK / CH;
      const long jp = j.j_plane / 8, wp = j.w_plane / 8;
      bf16x8 aa[2][CH][2], bb[2][CH][2];
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          aa[0][c][t] = srcJ[t * jp + c * 64];
          bb[0][c][t] = srcW[t * wp + c * 64];
        }
      f32x16 accl;
#pragma unroll
      for (int r = 0; r < 16; ++r) accl[r] = 0.f;
#pragma unroll
      for (int h = 0; h < NCH; ++h) {
        const int cur = h & 1;
        if (h + 1 < NCH) {
#pragma unroll
          for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
              aa[cur ^ 1][c][t] = srcJ[t * jp + ((h + 1) * CH + c) * 64];
              bb[cur ^ 1][c][t] = srcW[t * wp + ((h + 1) * CH + c) * 64];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const bf16x8 x[2] = {aa[cur][c][0], aa[cur][c][1]};
          const bf16x8 y[2] = {bb[cur][c][0], bb[cur][c][1]};
          mfma_h3(x, y, acc, accl);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += accl[r] * kF16LoInv;
    }
    // + bias, then a 4 x 4 transpose inside each lane quad (two DPP butterfly steps) so that
    // every lane holds 4 consecutive columns of one row: 16-byte write-through stores (a 4-byte
    // sc1 store is one fabric write each, ~6x the 16-byte store's time per byte)
    const int col = g * 32 + (lane & 31);
    const float bv = j.bias[col < j.V ? col : j.V - 1];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += bv;
    const int qi = lane & 3;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      float v[4] = {acc[4 * b], acc[4 * b + 1], acc[4 * b + 2], acc[4 * b + 3]};
      float t[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float o = dpp_f<kDppQuad1>(v[jj ^ 1]);
        t[jj] = ((jj ^ qi) & 1) ? o : v[jj];
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float o = dpp_f<kDppQuad2>(t[jj ^ 2]);
        v[jj] = ((jj ^ qi) & 2) ? o : t[jj];
      }
      // lane (hh, quad q, qi): row 8 b + 4 hh + qi, columns 4 q .. 4 q + 3 of the group
      const int row = m0 + 8 * b + 4 * (lane >> 5) + qi;
      const int c0 = g * 32 + 4 * ((lane & 31) >> 2);
      if (row < j.M)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(unsigned __attribute__((ext_vector_type(4))),
                               make_float4(v[0], v[1], v[2], v[3])),
            rso, (row * a.ldo + c0) * 4, 0, kCpolSc1);
    }
  }
  // ---- arrival: every wave's stores complete, then one ticket per block ----
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(a.cnt + rt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == nct - 1;
    if (last) __hip_atomic_store(a.cnt + rt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;

  // ---- the row tile's greedy step: wave w = stream 8 rt + w ----
  const int s = rt * 8 + wid;
  if (s >= a.S) return;
  const SearchState& st = a.st;
  const DecTable& dt = a.dt;
  const HotwordTables& hw = a.hw;
  const int V = j.V;
  const int T_s = a.enc_len[s];
  const int t0 = a.t_cur[s];
  if (t0 >= T_s) return;
  const int nf = T_s - t0 < F ? T_s - t0 : F;
  const int V4 = V >> 2;
  const int D = dt.D, d4 = D >> 2;
  const int base = s;  // Hmax = 1
  const int y1 = st.y1[base], y2 = st.y2[base];
  // rows in a 3-deep register ring (rows 0..2 loaded at once, row r + 3 once row r is done):
  // greedy needs the rows only up to the window's first emission, and with all four rows live
  // beside the emitting row's entropy work the wave would need more than 256 registers
  auto load_row = [&](float4 (&x)[Q], int r) {
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int i = lane + 64 * q;
      const int ii = i < V4 ? i : V4 - 1;
      const float4 v = __builtin_bit_cast(
          float4, __builtin_amdgcn_raw_buffer_load_b128(rso, ((s * F + r) * a.ldo + 4 * ii) * 4, 0,
                                                        kCpolSc1));
      x[q] = (r < nf && i < V4) ? v : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    }
  };
  float4 xr[3][Q];
  load_row(xr[0], 0);
  load_row(xr[1], 1);
  load_row(xr[2], 2);
  double lp = st.lp[base];
  // per row in frame order (greedy_spec steps A-D): statistics, the score before the frame
  // under the all-blank hypothesis (lf), the top-1; the first non-blank top-1 is the emission
  int fe = -1, tok = 0;
  float m1 = 0.f, m2 = 0.f, se = 1.f, ls = 0.f, lf = 0.f, e1 = 0.f, e3 = 0.f;
  double lpb = 0.0;
#pragma unroll
  for (int r = 0; r < F; ++r) {
    if (r >= nf) break;  // wave-uniform
    float4 (&x)[Q] = xr[r % 3];
    float rm1 = -INFINITY, rm2 = -INFINITY;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const float4 v = x[q];
      rm2 = fmaxf(rm2, fminf(rm1, v.x)); rm1 = fmaxf(rm1, v.x);
      rm2 = fmaxf(rm2, fminf(rm1, v.y)); rm1 = fmaxf(rm1, v.y);
      rm2 = fmaxf(rm2, fminf(rm1, v.z)); rm1 = fmaxf(rm1, v.z);
      rm2 = fmaxf(rm2, fminf(rm1, v.w)); rm1 = fmaxf(rm1, v.w);
    }
    wave_max2_dpp(rm1, rm2);
    float rse = 0.f;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      rse += __expf(x[q].x - rm1);
      rse += __expf(x[q].y - rm1);
      rse += __expf(x[q].z - rm1);
      rse += __expf(x[q].w - rm1);
    }
    rse = wave_sum_dpp(rse);
    const float rls = logf(rse);
    const float d0 = lane_f(x[0].x, 0) - rm1;  // blank = token 0 = lane 0's first element
    const float rlf = (float)lp;
    const float vmax = (0.f - rls) + rlf;
    int bq = 0x7fffffff;
#pragma unroll
    for (int q = Q - 1; q >= 0; --q) {
      const int i = 4 * (lane + 64 * q);
      const float4 v = x[q];
      const int c = (((v.x - rm1) - rls) + rlf == vmax) ? i
                  : (((v.y - rm1) - rls) + rlf == vmax) ? i + 1
                  : (((v.z - rm1) - rls) + rlf == vmax) ? i + 2
                  : (((v.w - rm1) - rls) + rlf == vmax) ? i + 3 : 0x7fffffff;
      bq = c < bq ? c : bq;
    }
    const int bm = wave_min_i_dpp(bq);
    const int best = bm < V ? bm : 0;
    if (best != 0) {  // the emission: this row's entropy terms (search_step_kernel's statistics)
      fe = r;
      tok = best;
      m1 = rm1;
      m2 = rm2;
      se = rse;
      ls = rls;
      lf = rlf;
      lpb = lp;
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const float vv[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float d = vv[c] - m1;
          const float e = __expf(d);
          e1 = (e > 0.f) ? fmaf(e, d, e1) : e1;
          e3 += __expf(d * (1.0f / 3.0f));
        }
      }
      break;
    }
    lp = (double)((d0 - rls) + rlf);
    if (r + 3 < F) load_row(xr[r % 3], r + 3);
  }
  const int t_new = t0 + (fe >= 0 ? fe + 1 : nf);
  if (fe >= 0) {
    e1 = wave_sum_dpp(e1);
    e3 = wave_sum_dpp(e3);
    if (lane == 0) {
      const float val = (0.f - ls) + lf;
      double score = (double)val;
      int nhw = st.hw[base];
      if (hw.num_states > 0 && tok != 2) {
        const int cls = hw.tok2cls[tok];
        if (cls < 0) {
          score += -hw.node_score[nhw];
          nhw = 0;
        } else {
          const long e = (long)nhw * hw.num_cls + cls;
          score += hw.delta[e];
          nhw = hw.next[e];
        }
      }
      const int nid = st.node_count[s];
      const long gi = (long)s * st.node_cap + nid;
      st.node_tok[gi] = tok;
      st.node_frame[gi] = t0 + fe;
      st.node_parent[gi] = st.node[base];
      st.node_lp[gi] = (double)val - lpb;
      st.node_stats[gi] = make_float4(ls - e1 / se, e3 * exp2f(-log2f(se) * (1.0f / 3.0f)),
                                      1.0f / se, __expf(m2 - m1) / se);
      st.node_count[s] = nid + 1;
      st.lp[base] = score;
      st.lpf[base] = 0;
      st.hash[base] = hash_push(st.hash[base], tok);
      st.len[base] = st.len[base] + 1;
      st.y2[base] = y1;
      st.y1[base] = tok;
      st.hw[base] = nhw;
      st.node[base] = nid;
    }
  } else if (lane == 0) {
    st.lp[base] = lp;  // the score after the window's nf blank frames
    st.lpf[base] = 0;
  }
  // the next window's rows and the new context's table row (issued once the window's rows are
  // dead: with them live beside these the wave would need more than 256 registers)
  const bool more = t_new < T_s;
  const int nf2 = T_s - t_new < F ? T_s - t_new : F;
  const int ny2 = fe >= 0 ? y1 : y2, ny1 = fe >= 0 ? tok : y1;
  float4 tv[2], ev[F][2];
  if (more) {
    const float4* tab4 = reinterpret_cast<const float4*>(dt.table + ((long)ny2 * dt.V + ny1) * D);
    const float4* enc4 = reinterpret_cast<const float4*>(dt.enc + (long)(dt.enc_off[s] + t_new) * D);
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int c4 = lane + 64 * jj < d4 ? lane + 64 * jj : d4 - 1;
      tv[jj] = tab4[c4];
#pragma unroll
      for (int f = 0; f < F; ++f) ev[f][jj] = enc4[(long)(f < nf2 ? f : 0) * d4 + c4];
    }
  }
  if (lane == 0) {
    a.t_cur[s] = t_new;
    if (more) atomicAdd(&a.active[a.parity], 1);
  }
  // ---- the next window's joiner input: J[s][f] = tanh(enc[t_new + f] + table[ny2, ny1]) ----
  if (!more) return;
#pragma unroll
  for (int jj = 0; jj < 2; ++jj) {
    const int c4 = lane + 64 * jj;
    if (c4 >= d4) continue;
#pragma unroll
    for (int f = 0; f < F; ++f)
      if (f < nf2) store_j4(dt, (long)s * F + f, 4 * c4, ev[f][jj], tv[jj]);
  }
}

void launch_joiner_greedy(const GreedyFusedArgs& a, hipStream_t st) {
  if (a.S <= 0) return;
  const JoinerPackedArgs& j = a.j;
  ZASR_REQUIRE(j.M == a.S * 4, "joiner_greedy: 4 window rows per stream");
  ZASR_REQUIRE(j.V % 4 == 0 && j.V <= 2048, "joiner_greedy: vocabulary a multiple of 4, <= 2048");
  ZASR_REQUIRE(a.ldo >= j.V && a.ldo % 32 == 0, "joiner_greedy: logits row stride");
  ZASR_REQUIRE(j.D == 256 || j.D == 512, "joiner_greedy: joiner dim must be 256 or 512");
  ZASR_REQUIRE(a.dt.D == j.D && a.dt.j_packed, "joiner_greedy: packed J of the joiner's dim");
  ZASR_REQUIRE(j.pieces == 0 || j.pieces == kPiecesF16, "joiner_greedy: bf16 or f16x3 operands");
  ZASR_REQUIRE((long)j.M * a.ldo * 4 < 0x7fffffffL, "joiner_greedy: logits beyond 2 GB");
  const dim3 grid(cdiv(j.V, 256), cdiv(a.S, 8));
  const int qk = j.D / 16;
#define ZASR_JG(QKV, FMTV, QV) \
  ZASR_LAUNCH((joiner_greedy_kernel<QKV, FMTV, QV>), grid, dim3(512), 0, st, a)
  if (j.pieces == kPiecesF16) {
    if (j.V <= 512) { if (qk == 16) ZASR_JG(16, 1, 2); else ZASR_JG(32, 1, 2); }
    else { if (qk == 16) ZASR_JG(16, 1, 8); else ZASR_JG(32, 1, 8); }
  } else {
    if (j.V <= 512) { if (qk == 16) ZASR_JG(16, 0, 2); else ZASR_JG(32, 0, 2); }
    else { if (qk == 16) ZASR_JG(16, 0, 8); else ZASR_JG(32, 0, 8); }
  }
#undef ZASR_JG
}

// --------------------------------------------------------------------------------------
// finalize (:1142-1148), length-normalised pick (:1151), backtrack the emission chain.
// One wave per stream: the stream's parent pointers are staged into LDS by coalesced loads
// (one HBM round trip instead of one per emission: a thread walking the chain in global
// memory paid ~1 us per token), lane 0 walks the chain in LDS recording the node of every
// output position, and the 64 lanes gather the nodes' fields into the outputs.  A stream
// with more nodes than the stage holds walks in global memory as before.
constexpr int kFinalStage = 8192;  // nodes staged per stream (32 KB of parents)
constexpr int kFinalPath = 2048;   // output positions recorded in LDS (8 KB)
__global__ __launch_bounds__(64) void search_final_kernel(SearchState st, int S, int Hmax,
                                                          HotwordTables hw, int out_cap,
                                                          int* out_tok, int* out_frame,
                                                          double* out_lp, float4* out_stats,
                                                          int* out_count) {
  __shared__ int sPar[kFinalStage];
  __shared__ int sPath[kFinalPath + 1];
  const int s = blockIdx.x, lane = threadIdx.x;
  if (s >= S) return;
  const int base = s * Hmax;
  const int n = st.nh[s];
  int best = 0;
  double best_v = -INFINITY;
  for (int h = 0; h < n; ++h) {  // every lane the same pick (uniform loads)
    double lp = st.lp[base + h];
    if (hw.num_states > 0) lp += -hw.node_score[st.hw[base + h]];
    double v = lp / (double)(st.len[base + h] > 1 ? st.len[base + h] : 1);
    if (h == 0 || v > best_v) {
      best_v = v;
      best = h;
    }
  }
  const long pool = (long)s * st.node_cap;
  const int nodes = st.node_count[s];
  const int start = st.node[base + best];
  if (nodes > kFinalStage) {  // the chain walked in global memory (one lane)
    if (lane != 0) return;
    int cnt = 0;
    for (int nd = start; nd >= 0; nd = st.node_parent[pool + nd]) ++cnt;
    if (cnt > out_cap) cnt = out_cap;
    int pos = cnt - 1;
    for (int nd = start; nd >= 0 && pos >= 0; nd = st.node_parent[pool + nd], --pos) {
      const long g = pool + nd, o = (long)s * out_cap + pos;
      out_tok[o] = st.node_tok[g];
      out_frame[o] = st.node_frame[g];
      out_lp[o] = st.node_lp[g];
      out_stats[o] = st.node_stats[g];
    }
    out_count[s] = cnt;
    return;
  }
  for (int i = lane; i < nodes; i += 64) sPar[i] = st.node_parent[pool + i];
  __syncthreads();
  // lane 0: the chain's length, then its nodes newest first into sPath (the newest out_cap
  // nodes when the chain is longer, as the two-walk form kept)
  if (lane == 0) {
    int cnt = 0;
    for (int nd = start; nd >= 0; nd = sPar[nd]) ++cnt;
    if (cnt > out_cap) cnt = out_cap;
    sPath[kFinalPath] = cnt;
    if (cnt <= kFinalPath) {
      int pos = cnt - 1;
      for (int nd = start; nd >= 0 && pos >= 0; nd = sPar[nd], --pos) sPath[pos] = nd;
    }
  }
  __syncthreads();
  const int cnt = sPath[kFinalPath];
  if (cnt <= kFinalPath) {
    for (int pos = lane; pos < cnt; pos += 64) {
      const long g = pool + sPath[pos], o = (long)s * out_cap + pos;
      out_tok[o] = st.node_tok[g];
      out_frame[o] = st.node_frame[g];
      out_lp[o] = st.node_lp[g];
      out_stats[o] = st.node_stats[g];
    }
  } else if (lane == 0) {
    int pos = cnt - 1;
    for (int nd = start; nd >= 0 && pos >= 0; nd = sPar[nd], --pos) {
      const long g = pool + nd, o = (long)s * out_cap + pos;
      out_tok[o] = st.node_tok[g];
      out_frame[o] = st.node_frame[g];
      out_lp[o] = st.node_lp[g];
      out_stats[o] = st.node_stats[g];
    }
  }
  if (lane == 0) out_count[s] = cnt;
}

void launch_search_final(const SearchState& s, int S, int Hmax, const HotwordTables& hw,
                         int out_cap, int* out_tok, int* out_frame, double* out_lp,
                         float4* out_stats, int* out_count, hipStream_t st) {
  if (S <= 0) return;
  ZASR_LAUNCH(search_final_kernel, dim3(S), dim3(64), 0, st, s, S, Hmax, hw, out_cap, out_tok,
              out_frame, out_lp, out_stats, out_count);
}

}  // namespace zasr
