// Attention kernels of the Zipformer2 encoder (icefall zipformer.py
// RelPositionMultiheadAttentionWeights / SelfAttention / NonlinAttention, 3P; the reference
// runs them inside the exported encoder, core/asr_engine.py:1045-1049): the flash-style
// kernel below (modes 0-3), and the kernels of the unfused NonlinAttention route:
//
//   z = (A0 @ (tanh(s) * x)) * y,   (s, x, y) = chunk(in_proj(src), 3),
//   A0 = softmax over keys of head 0 of RelPositionMultiheadAttentionWeights.
//
// The product A0 @ t1 is a per-sequence GEMM with K = L (up to ~1700 keys): it runs on the
// bf16 MFMA GEMM (gemm.hip, one z-slice per sequence) with
//   A = A0 in bf16, [L][L32] per sequence (L32 = L rounded up to 32, columns >= L zero),
//   B = t1 transposed in bf16, [hid][R32] (sequence b in columns [o32_b, o32_b + L32_b), zero
//       padded), i.e. the [N][K] "weight" layout the GEMM streams with 16-byte loads,
// and the `* y` factor in its epilogue.  The kernels here produce A0 and t1^T.
#include <mutex>
#include <string>
#include <type_traits>
#include <unordered_map>

#include "common.h"
#include "gemm.h"
#include "gemm_dev.h"
#include "kernels.h"

namespace zasr {


// =====================================================================================
// bf16-mode attention (RelPositionMultiheadAttentionWeights + SelfAttention, icefall
// zipformer.py, 3P), flash style: scores are recomputed where they are consumed and never
// reach HBM except head 0's normalised weights (NonlinAttention's GEMM operand).
//
// Block = 4 waves = 128 queries of one (sequence, head); wave w owns queries
// i0 + 32 w + (lane & 31) and walks every 32-key block of the sequence.  Per key block the
// block stages K (32 keys x 32 dims) and V^T (12 dims x 32 keys, permuted into the
// accumulator order of the scores) in LDS once for all 4 waves, double-buffered with the
// next block's global loads in registers.  The positional rows R[x] (x = j - i) the block
// touches (L + 127 of them) are staged once at the start.
//
//   S^T = K Q^T     v_mfma_f32_32x32x16_bf16: lane = query, registers = 16 keys
//         + p_i . R[j - i]
//   P^T = exp2(S^T - c_i)     (log2 domain: q and p carry log2 e from attn_in's weights)
//   O^T += V^T P^T            (the accumulator registers are the MFMA k-slots as they stand)
//
// MODE 0 (W0): head 0, pass 1 = row statistics, pass 2 = normalised weights in bf16.
// MODE 1 (SA online): running max / sum, O rescaled when the max moves; writes the output
//   and the row statistic c_i = max + log2(sum) for the second self-attention.
// MODE 2 (SA stats): c_i from MODE 1, P normalised directly.
// =====================================================================================
namespace {
constexpr int kKLd = 40;  // LDS row stride (bf16) of the K / V^T images: 80 B
constexpr int kPosPad = 160;  // staged positional rows beyond L (the last key block's tail)

__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// packed f32 pair: one v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32 does two lanes' worth of
// f32 work per issue (the kernels below are VALU-bound: SQ_ACTIVE_INST_VALU ~0.75 of SIMD
// cycles, profiles/r03/attn_pmc/)
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }

// ---- the f16x3 mode's one-accumulator products (FMT 1) ----
// x = (x0, x1) = fp16 pieces (hi, lo 2^11) of the A operand (V^T or t1^T, staged in LDS); the
// B operand (the weights P^T <= 1) carries three pieces: ys = hi 2^11 (exact in fp16), yh = hi,
// yl = lo 2^11.  acc (scaled by 2^11) += x1 yh + x0 yl + x0 ys, smallest terms first:
// the same three fp16 MFMAs as the two-accumulator form on one accumulator, so no lo
// accumulator to hold, rescale and fold back (16 VGPRs per output fragment)
typedef _Float16 f16x8a __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void mfma_h3s(const bf16x8 (&x)[2], const f16x8a& ys, const f16x8a& yh,
                                         const f16x8a& yl, f32x16& acc) {
  const f16x8a x0 = __builtin_bit_cast(f16x8a, x[0]), x1 = __builtin_bit_cast(f16x8a, x[1]);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x1, yh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, yl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(x0, ys, acc, 0, 0, 0);
}

// pieces of 8 weights from e = 2^11 p (the exp2 argument carries the + 11; p <= 1, e <= 2048):
// ys = fp16(e), yh = ys 2^-11, yl = fp16(e - ys) = (p - yh) 2^11 (e - ys is exact in f32)
__device__ __forceinline__ void split_e8(const float* e, f16x8a& ys, f16x8a& yh, f16x8a& yl) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 sp, lp;
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const f16x2 h2 = {(_Float16)e[q], (_Float16)e[q + 1]};
    const unsigned hs = __builtin_bit_cast(unsigned, h2);
    // lo pieces e - fp16(e), exact in f32 and rounded once to fp16, by v_fma_mix (the fp16
    // operand widened inside the instruction): 2 instructions a pair where widen / subtract /
    // pack take 4 (the compiler does not form it from the C expression)
    unsigned lo;
    asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]\n\t"
        "v_fma_mixhi_f16 %0, %1, -1.0, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
        : "=&v"(lo) : "v"(hs), "v"(e[q]), "v"(e[q + 1]));
    sp[q / 2] = hs;
    lp[q / 2] = lo;
  }
  ys = __builtin_bit_cast(f16x8a, sp);
  yl = __builtin_bit_cast(f16x8a, lp);
  const _Float16 k = (_Float16)(1.f / 2048.f);
  yh = ys * (f16x8a){k, k, k, k, k, k, k, k};
}

}  // namespace

// NP = 1: bf16 storage (the bf16 mode).  NP = 2 / 3: q / k / p / v / out / the head-0 weights
// are f32 and every MFMA operand is split into NP bf16 pieces (x = p0 + p1 [+ p2]); a product
// is the sum of the piece products p_u q_v with u + v < NP (3 / 6 MFMAs where the bf16 mode
// issues one): near-f32 (NP = 2) / f32-quality (NP = 3) scores and outputs at bf16 MFMA rates
// (the bf16x3 / bf16x6 modes).  In these modes q and p carry no log2(e) factor: the score is
// scaled into the log2 domain after the positional term.
// FMT 1 (the f16x3 mode, NP = 2): the pieces are fp16 hi + lo * 2^-11 (gemm_dev.h split_h8)
// and every product is hi*hi + (hi*lo + lo*hi) * 2^-11 on fp16 MFMAs: the scores with the lo
// products in a second accumulator (combined per key block), the PV products in the
// one-accumulator form (mfma_h3s): the weights enter as e = 2^11 p straight from the exp2
// (p <= 1, so e's hi piece is exact in fp16), O accumulates 2^11-scaled on one register set
// and the row sum, which carries the same 2^11, cancels it.
// MODE 3 (NF = value fragments per block): NonlinAttention, z = (A0 @ t1) * y, in ONE online
// pass over head 0: running max / sum as in mode 1, the unnormalised weights P^T (<= 1; the
// score registers as they stand) multiplied into V^T = this block's NF x 32 rows of t1t
// (grid.z = chunks of hid), the value accumulators rescaled when the max moves, 1 / sum and
// * y in the epilogue -- head 0's L x L weights never reach HBM (mode 0 + the z-sliced GEMM
// wrote and read them).  bf16 mode: y / z bf16; f16x3 (FMT 1): two fp16 pieces of the weights
// and of t1, hi / lo value accumulators, y / z f32.
template <int MODE, int NP, int FMT = 0, int NF = 1>
__global__ __launch_bounds__(256) void attn_flash_kernel(AttnFlashArgs a) {
  constexpr bool SPLIT = NP > 1;
  // FMT 1: the PV products in the one-accumulator form (mode 0 has no PV products)
  constexpr bool P1 = FMT == 1;
  static_assert(FMT == 0 || NP == 2, "fp16 pieces: NP = 2");
  static_assert(MODE != 3 || NP == 1 || (NP == 2 && FMT == 1),
                "fused NonlinAttention: the bf16 and f16x3 modes");
  constexpr bool W0 = MODE == 0 || MODE == 3;  // head 0
  using T = typename std::conditional<SPLIT, float, __bf16>::type;
  // positional rows of this head, x = xlo + t for t < L + kPosPad, one plane per pos dim
  // (structure of arrays: the rows of two adjacent keys are adjacent floats in each plane,
  // so a ds_read2_b32 puts them into the register pair a packed FMA takes)
  extern __shared__ float sPos[];
  __shared__ __attribute__((aligned(16))) __bf16 sK[NP][2][32 * kKLd];
  __shared__ __attribute__((aligned(16))) __bf16 sVt[NP][2][12 * kKLd];
  // mode 3: V^T = t1t rows [fz NF 32, +NF 32) x 32 keys, keys permuted like sVt's
  __shared__ __attribute__((aligned(16))) __bf16 sVn[NP][2][MODE == 3 ? NF * 32 * kKLd : 8];
  const int b = blockIdx.y;
  const int h = W0 ? 0 : blockIdx.z;
  const int fz = MODE == 3 ? blockIdx.z : 0;
  const int r0 = a.row_off[b];
  const int L = a.row_off[b + 1] - r0;
  const int i0b = blockIdx.x * 128;
  if (i0b >= L) return;
  const int H = a.H;
  const long ldq = 68L * H;
  const long ldv = 12L * H;
  const T* qkp = reinterpret_cast<const T*>(a.qkp);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int c = lane & 31, h2 = lane >> 5;
  const int i0 = i0b + 32 * wid;
  const bool live = i0 < L;  // wave-uniform
  const int i = i0 + c;
  const int ic = i < L ? i : L - 1;
  constexpr float kSc = SPLIT ? 1.4426950408889634f : 1.f;  // log2(e) applied in-kernel
  // FMT 1: the weights enter the PV products as e = 2^11 p (exp2 argument + 11); the row sum
  // then carries 2^11, which the normalisation cancels (mode 1's statistic subtracts the 11)
  constexpr float kE = P1 ? 11.f : 0.f;

  // ---- positional rows: x in [xlo, xlo + L + kPosPad) ----
  {
    const int xlo = -(i0b + 127);
    const int n = L + kPosPad;
    const int rmax = 2 * a.pmax - 2;
    for (int t = tid; t < n; t += 256) {
      int row = xlo + t + a.pmax - 1;
      row = row < 0 ? 0 : (row > rmax ? rmax : row);
      const float4 v = *reinterpret_cast<const float4*>(a.pos_tab + (long)row * 4 * H + 4 * h);
      if constexpr (SPLIT) {
        sPos[t] = v.x;
        sPos[n + t] = v.y;
        sPos[2 * n + t] = v.z;
        sPos[3 * n + t] = v.w;
      } else {
        // bf16 mode: the rows in bf16 (8 B), consumed by v_dot2_f32_bf16 against the bf16 p_i
        const bf16x4 w = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
        reinterpret_cast<bf16x4*>(sPos)[t] = w;
      }
    }
  }
  // ---- this lane's query (dims 8 h2 .. +8 and 16 + 8 h2 .. +8) and positional query ----
  const T* qrow = qkp + (long)(r0 + ic) * ldq + 32 * h;
  bf16x8 qf0[NP], qf1[NP];
  float4 pq = make_float4(0.f, 0.f, 0.f, 0.f);
  bf16x2 pq01, pq23;  // bf16 mode: p_i as two bf16 pairs for v_dot2_f32_bf16
  if constexpr (SPLIT) {
    float v0[8], v1[8];
    *reinterpret_cast<float4*>(&v0[0]) = *reinterpret_cast<const float4*>(qrow + 8 * h2);
    *reinterpret_cast<float4*>(&v0[4]) = *reinterpret_cast<const float4*>(qrow + 8 * h2 + 4);
    *reinterpret_cast<float4*>(&v1[0]) = *reinterpret_cast<const float4*>(qrow + 16 + 8 * h2);
    *reinterpret_cast<float4*>(&v1[4]) = *reinterpret_cast<const float4*>(qrow + 20 + 8 * h2);
    split_fx<FMT, NP>(v0, qf0);
    split_fx<FMT, NP>(v1, qf1);
    pq = *reinterpret_cast<const float4*>(qkp + (long)(r0 + ic) * ldq + 64 * H + 4 * h);
  } else {
    qf0[0] = *reinterpret_cast<const bf16x8*>(qrow + 8 * h2);
    qf1[0] = *reinterpret_cast<const bf16x8*>(qrow + 16 + 8 * h2);
    const bf16x4 pv = *reinterpret_cast<const bf16x4*>(qkp + (long)(r0 + ic) * ldq + 64 * H + 4 * h);
    pq01 = (bf16x2){pv[0], pv[1]};
    pq23 = (bf16x2){pv[2], pv[3]};
  }
  // pos index of (this query, key j0 + jr): j0 + jr - 32 wid - c + 127
  const int pbase = 127 - 32 * wid - c;

  const int nkb = (L + 31) / 32;
  // staging roles: threads 0..127 load K (key tid>>2, 8 dims 8 (tid&3)); threads 128..223
  // load V (key (tid-128)/3, 4 dims (tid-128)%3); MODE 0 needs no V
  const T* kbase = qkp + (long)r0 * ldq + 32 * H + 32 * h;
  const T* vbase = W0 ? nullptr : reinterpret_cast<const T*>(a.v) + (long)r0 * ldv + 12 * h;
  const int vt = tid - 128;
  const int vkey = vt / 3, vq = vt - 3 * (vt / 3);
  // two register sets: key block kb + 2's global loads are in flight while block kb is
  // computed and block kb + 1 (loaded one block earlier) goes to LDS, so the loads have two
  // blocks of compute to land in (one block was not enough to cover their latency)
  bf16x8 kv[2];  // bf16 mode: K threads' 8 dims, or V threads' 4 dims in elements 0..3
  // split modes: f32 staging registers; K rows (threads < 128) use both, V rows the first
  float4 stg0[2], stg1[2];
  // every thread issues the same loads whatever its role (threads without one re-read a K
  // row), so the wait before storing a set can count the newer set's loads still in flight
  // (divergent load sites made the compiler wait for everything)
  const bool vrole = !W0 && vt >= 0 && vt < 96;
  auto gload = [&](int kb, auto set) {
    constexpr int S = decltype(set)::value;
    const int j0 = kb * 32;
    int j = j0 + (vrole ? vkey : ((tid >> 2) & 31));
    j = j < L ? j : L - 1;
    const T* src = vrole ? vbase + (long)j * ldv + 4 * vq : kbase + (long)j * ldq + 8 * (tid & 3);
    if constexpr (SPLIT) {
      stg0[S] = *reinterpret_cast<const float4*>(src);
      stg1[S] = *reinterpret_cast<const float4*>(src + (vrole ? 0 : 4));
    } else {
      // a V thread reads 8 dims of which it keeps 4 (the row tail past the head is in bounds:
      // the next head's or, for the very last row, the workspace's slack)
      kv[S] = *reinterpret_cast<const bf16x8*>(src);
    }
  };
  auto sstore = [&](int buf, auto set) {
    constexpr int S = decltype(set)::value;
    if (tid < 128) {
      __bf16* d = &sK[0][buf][(tid >> 2) * kKLd + 8 * (tid & 3)];
      if constexpr (SPLIT) {
        const float v[8] = {stg0[S].x, stg0[S].y, stg0[S].z, stg0[S].w,
                            stg1[S].x, stg1[S].y, stg1[S].z, stg1[S].w};
        bf16x8 pc[NP];
        split_fx<FMT, NP>(v, pc);
#pragma unroll
        for (int t = 0; t < NP; ++t) *reinterpret_cast<bf16x8*>(d + t * 2 * 32 * kKLd) = pc[t];
      } else {
        *reinterpret_cast<bf16x8*>(d) = kv[S];
      }
    } else if (!W0 && vt < 96) {
      // key jj sits in score register r = (jj&3) + 4 (jj>>3) of lane half (jj>>2)&1, which
      // the PV MFMA m = r >> 3 takes in k-slot 8 half + (r & 7)
      const int jj = vkey;
      const int r = (jj & 3) + 4 * (jj >> 3);
      const int slot = 16 * (r >> 3) + 8 * ((jj >> 2) & 1) + (r & 7);
      if constexpr (SPLIT) {
        auto put = [&](int e, float rr) {
          if constexpr (FMT == 1) {
            const _Float16 hh = (_Float16)rr;
            sVt[0][buf][(4 * vq + e) * kKLd + slot] = __builtin_bit_cast(__bf16, hh);
            sVt[1][buf][(4 * vq + e) * kKLd + slot] =
                __builtin_bit_cast(__bf16, (_Float16)((rr - (float)hh) * kF16Lo));
          } else {
#pragma unroll
            for (int t = 0; t < NP; ++t) {
              const __bf16 hh = (__bf16)rr;
              sVt[t][buf][(4 * vq + e) * kKLd + slot] = hh;
              if (t + 1 < NP) rr -= (float)hh;
            }
          }
        };
        put(0, stg0[S].x);
        put(1, stg0[S].y);
        put(2, stg0[S].z);
        put(3, stg0[S].w);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) sVt[0][buf][(4 * vq + e) * kKLd + slot] = kv[S][e];
      }
    }
  };
  // mode 3: V^T staging, NF 32 rows x 32 keys per key block = NF * 128 16-byte pieces (8 keys
  // of one t1 row), NV per thread, loaded with the K rows' cadence (two sets in flight)
  constexpr int NV = MODE == 3 ? (NF * 128 + 255) / 256 : 1;
  bf16x8 v3[2][NV][NP];  // (NP = 2: t1t's hi / lo piece images, hid x ldt apart)
  const __bf16* t1b = MODE == 3 ? reinterpret_cast<const __bf16*>(a.t1t) + a.o8[b] : nullptr;
  auto gload3 = [&](int kb, auto set) {
    constexpr int S = decltype(set)::value;
    if constexpr (MODE == 3) {
      const int j0 = (kb < nkb ? kb : nkb - 1) * 32;  // (clamped: the tail loads re-read)
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int e = tid + 256 * u;
        const int dr = (e >> 2) < NF * 32 ? (e >> 2) : NF * 32 - 1;
        int dg = fz * NF * 32 + dr;
        dg = dg < a.hid ? dg : a.hid - 1;
#pragma unroll
        for (int t = 0; t < NP; ++t)
          v3[S][u][t] = *reinterpret_cast<const bf16x8*>(t1b + ((long)t * a.hid + dg) * a.ldt + j0 + 8 * (e & 3));
      }
    }
  };
  auto sstore3 = [&](int buf, auto set) {
    constexpr int S = decltype(set)::value;
    if constexpr (MODE == 3) {
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const int e = tid + 256 * u;
        if (NV * 256 == NF * 128 || e < NF * 128) {
          const int dr = e >> 2, g8 = e & 3;
          // keys 8 g8 + q: q < 4 -> slot s0 + q, q >= 4 -> s0 + 8 + (q - 4) (see sstore)
          const int s0 = 16 * (g8 >> 1) + 4 * (g8 & 1);
          const bool live_row = fz * NF * 32 + dr < a.hid;  // rows past hid stay zero
#pragma unroll
          for (int t = 0; t < NP; ++t) {
            bf16x8 v = v3[S][u][t];
            if (!live_row) v = (bf16x8){};
            __bf16* d = &sVn[t][buf][dr * kKLd + s0];
            *reinterpret_cast<bf16x4*>(d) = (bf16x4){v[0], v[1], v[2], v[3]};
            *reinterpret_cast<bf16x4*>(d + 8) = (bf16x4){v[4], v[5], v[6], v[7]};
          }
        }
      }
    }
  };
  // scores of key block kb (log2 domain), keys >= L masked to -inf
  auto scores = [&](int kb, int buf, f32x16& s) {
    const int j0 = kb * 32;
    bf16x8 k0[NP], k1[NP];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      k0[t] = *reinterpret_cast<const bf16x8*>(&sK[t][buf][c * kKLd + 8 * h2]);
      k1[t] = *reinterpret_cast<const bf16x8*>(&sK[t][buf][c * kKLd + 16 + 8 * h2]);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s[r] = 0.f;
    if constexpr (FMT == 1) {
      // (the scores keep two accumulators: their one-accumulator form needs |q| < 32 and
      // measured slower in modes 1 / 2)
      f32x16 sl;
#pragma unroll
      for (int r = 0; r < 16; ++r) sl[r] = 0.f;
      mfma_h3(k0, qf0, s, sl);
      mfma_h3(k1, qf1, s, sl);
#pragma unroll
      for (int r = 0; r < 16; ++r) s[r] += sl[r] * kF16LoInv;
    } else {
      s = mfma_split<NP>(k0, qf0, s);
      s = mfma_split<NP>(k1, qf1, s);
    }
    const int pb = j0 + pbase;
    // positional term p_i . R[j - i] for the key pair (r, r + 1) = keys (jr, jr + 1) as packed
    // FMAs: the same fma chain per score as scalar fmaf, half the VALU issues
    if constexpr (!SPLIT) {
      // bf16 mode: p_i . R[j - i] as two bf16 dot products per score (8 LDS bytes a score
      // instead of 16: the kernels are bound by LDS bandwidth, profiles/r03/attn_pmc/)
      const bf16x4* pr = reinterpret_cast<const bf16x4*>(sPos) + pb;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jr = (r & 3) + 8 * (r >> 2) + 4 * h2;
        const bf16x4 w = pr[jr];
        s[r] = __builtin_amdgcn_fdot2_f32_bf16(pq23, (bf16x2){w[2], w[3]},
                                               __builtin_amdgcn_fdot2_f32_bf16(pq01, (bf16x2){w[0], w[1]}, s[r], false),
                                               false);
      }
    } else {
    const f32x2 qx = {pq.x, pq.x}, qy = {pq.y, pq.y}, qz = {pq.z, pq.z}, qw = {pq.w, pq.w};
    const int np = L + kPosPad;
    const float* px = sPos + pb;
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const int jr = (r & 3) + 8 * (r >> 2) + 4 * h2;
      f32x2 ps = {s[r], s[r + 1]};
      ps = pk_fma(qx, (f32x2){px[jr], px[jr + 1]}, ps);
      ps = pk_fma(qy, (f32x2){px[np + jr], px[np + jr + 1]}, ps);
      ps = pk_fma(qz, (f32x2){px[2 * np + jr], px[2 * np + jr + 1]}, ps);
      ps = pk_fma(qw, (f32x2){px[3 * np + jr], px[3 * np + jr + 1]}, ps);
      ps *= (f32x2){kSc, kSc};
      s[r] = ps.x;
      s[r + 1] = ps.y;
    }
    }
    if (j0 + 32 > L) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int jr = (r & 3) + 8 * (r >> 2) + 4 * h2;
        s[r] = j0 + jr < L ? s[r] : -INFINITY;
      }
    }
  };

  // ---- key-block loop(s) ----
  float m = -INFINITY, l = 0.f, cst = 0.f;
  if constexpr (MODE == 2) cst = a.stats_in[(long)(r0 + ic) * H + h];
  f32x16 o;  // (P1: scaled by 2^11, the weights entering as e = 2^11 p)
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = 0.f;
  // V^T fragments of the PV MFMAs; value dims d >= 12 (lanes c >= 12) stay zero
  bf16x8 vf[2][NP];
#pragma unroll
  for (int mm = 0; mm < 2; ++mm)
#pragma unroll
    for (int t = 0; t < NP; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) vf[mm][t][e] = (__bf16)0.f;

  constexpr int NPASS = MODE == 0 ? 2 : 1;
  // mode 3: O^T per 32-row value fragment
  f32x16 o3[MODE == 3 ? NF : 1];
#pragma unroll
  for (int f = 0; f < (MODE == 3 ? NF : 1); ++f)
#pragma unroll
    for (int r = 0; r < 16; ++r) o3[f][r] = 0.f;
  T* const a0 = MODE == 0 ? reinterpret_cast<T*>(a.attn) + a.a_off[b] : nullptr;
  // (mode 3: both passes unrolled, so the V^T staging and o3 exist in pass 2's code only)
  constexpr int kPassUnroll = MODE == 3 ? 2 : 1;
#pragma unroll kPassUnroll
  for (int pass = 0; pass < NPASS; ++pass) {
    constexpr bool vp = MODE == 3;  // mode 3's V^T staging
    if (W0 && pass == 1) {
      // row statistic from the two lane halves (same query, disjoint keys)
      const float mo = __shfl_xor(m, 32, 64), lo = __shfl_xor(l, 32, 64);
      const float M = fmaxf(m, mo);
      const float Ls = l * fexp2(m - M) + lo * fexp2(mo - M);
      cst = M + __log2f(Ls);
    }
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    gload(0, I0{});
    if (vp) gload3(0, I0{});
    if (nkb > 1) {
      gload(1, I1{});
      if (vp) gload3(1, I1{});
    }
    __syncthreads();  // previous pass's readers are done with buffer 0 (and sPos is staged)
    sstore(0, I0{});
    if (vp) sstore3(0, I0{});
    __syncthreads();
    // one key block: its loads went out two blocks ago (set S), block kb + 2's go out now
    // into the same set, block kb + 1 (set 1 - S) is stored for the next step
    auto block = [&](int kb, auto set) {
      constexpr int S = decltype(set)::value;
      const int cur = kb & 1;
      gload(kb + 2, set);  // unconditional (clamped rows past the end): see gload
      if (vp) gload3(kb + 2, set);
      if (live) {
        f32x16 s;
        scores(kb, cur, s);
        if constexpr (MODE == 3) {
          // one pass, online: running max / sum as mode 1, O rescaled when the max moves, the
          // unnormalised weights (<= 1) in the MFMA, 1 / sum in the epilogue
          float bm = s[0];
#pragma unroll
          for (int r = 1; r < 16; ++r) bm = fmaxf(bm, s[r]);
          bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
          const float mn = fmaxf(m, bm);
          if (__any(mn > m)) {
            const float sc = fexp2(m - mn);  // m = -inf -> 0
#pragma unroll
            for (int f = 0; f < NF; ++f)
#pragma unroll
              for (int r = 0; r < 16; r += 2) {
                const f32x2 v = (f32x2){o3[f][r], o3[f][r + 1]} * (f32x2){sc, sc};
                o3[f][r] = v.x;
                o3[f][r + 1] = v.y;
              }
            l *= sc;
            m = mn;
          }
          const f32x2 nm = {kE - m, kE - m};
          f32x2 acc = {0.f, 0.f};
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            const f32x2 dd = (f32x2){s[r], s[r + 1]} + nm;
            s[r] = fexp2(dd.x);
            s[r + 1] = fexp2(dd.y);
            acc += (f32x2){s[r], s[r + 1]};
          }
          l += acc.x + acc.y;
#pragma unroll
          for (int mm = 0; mm < 2; ++mm) {
            bf16x8 pf[NP];
            f16x8a ps3, ph3, pl3;  // P1: the weights' three pieces
            if constexpr (P1) {
              float ev[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) ev[q] = s[8 * mm + q];
              split_e8(ev, ps3, ph3, pl3);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) pf[0][q] = (__bf16)s[8 * mm + q];
            }
#pragma unroll
            for (int f = 0; f < NF; ++f) {
              bf16x8 vf3[NP];
#pragma unroll
              for (int t = 0; t < NP; ++t)
                vf3[t] = *reinterpret_cast<const bf16x8*>(&sVn[t][cur][(f * 32 + c) * kKLd + 16 * mm + 8 * h2]);
              if constexpr (P1)
                mfma_h3s(vf3, ps3, ph3, pl3, o3[f]);
              else
                o3[f] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf3[0], pf[0], o3[f], 0, 0, 0);
            }
          }
        } else if constexpr (MODE == 0) {
          if (pass == 0) {
            float bm = s[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) bm = fmaxf(bm, s[r]);
            const float mn = fmaxf(m, bm);
            if (mn != -INFINITY) {  // a lane half can see only masked keys (L <= 4)
              const f32x2 nm = {-mn, -mn};
              f32x2 acc = {0.f, 0.f};
#pragma unroll
              for (int r = 0; r < 16; r += 2) {
                const f32x2 d = (f32x2){s[r], s[r + 1]} + nm;
                acc += (f32x2){fexp2(d.x), fexp2(d.y)};
              }
              l = l * fexp2(m - mn) + (acc.x + acc.y);
              m = mn;
            }
          } else if (i < L) {
            // row stride L32: the key blocks cover [0, L32) exactly, keys >= L write zeros
            const int L32 = (L + 31) & ~31;
            const int j0 = kb * 32;
            T* dst = a0 + (long)i * L32 + j0 + 4 * h2;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              if constexpr (SPLIT) {
                float4 v;
                v.x = fexp2(s[4 * g + 0] - cst);
                v.y = fexp2(s[4 * g + 1] - cst);
                v.z = fexp2(s[4 * g + 2] - cst);
                v.w = fexp2(s[4 * g + 3] - cst);
                *reinterpret_cast<float4*>(dst + 8 * g) = v;
              } else {
                bf16x4 v;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = (__bf16)fexp2(s[4 * g + e] - cst);
                *reinterpret_cast<bf16x4*>(dst + 8 * g) = v;
              }
            }
          }
        } else {
          if constexpr (MODE == 1) {
            float bm = s[0];
#pragma unroll
            for (int r = 1; r < 16; ++r) bm = fmaxf(bm, s[r]);
            bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
            const float mn = fmaxf(m, bm);
            if (__any(mn > m)) {
              const float sc = fexp2(m - mn);  // m = -inf -> 0
              // o[8..15] are rows 16..31 of O^T: no value dims there (d < 12), never read
#pragma unroll
              for (int r = 0; r < 8; r += 2) {
                const f32x2 v = (f32x2){o[r], o[r + 1]} * (f32x2){sc, sc};
                o[r] = v.x;
                o[r + 1] = v.y;
              }
              l *= sc;
              m = mn;
            }
            const f32x2 nm = {kE - m, kE - m};
            f32x2 acc = {0.f, 0.f};
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const f32x2 d = (f32x2){s[r], s[r + 1]} + nm;
              s[r] = fexp2(d.x);
              s[r + 1] = fexp2(d.y);
              acc += (f32x2){s[r], s[r + 1]};
            }
            l += acc.x + acc.y;
          } else {
            const f32x2 nc = {kE - cst, kE - cst};
#pragma unroll
            for (int r = 0; r < 16; r += 2) {
              const f32x2 d = (f32x2){s[r], s[r + 1]} + nc;
              s[r] = fexp2(d.x);
              s[r + 1] = fexp2(d.y);
            }
          }
#pragma unroll
          for (int mm = 0; mm < 2; ++mm) {
            bf16x8 pf[NP];
            f16x8a ps3, ph3, pl3;  // P1: the weights' three pieces
            if constexpr (P1) {
              float ev[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) ev[q] = s[8 * mm + q];
              split_e8(ev, ps3, ph3, pl3);
            } else {
#pragma unroll
              for (int q = 0; q < 8; ++q) {
                float r = s[8 * mm + q];
#pragma unroll
                for (int t = 0; t < NP; ++t) {
                  const __bf16 hh = (__bf16)r;
                  pf[t][q] = hh;
                  if (t + 1 < NP) r -= (float)hh;
                }
              }
            }
            if (c < 12) {  // lanes 12..31 keep the zeros set before the loop
#pragma unroll
              for (int t = 0; t < NP; ++t)
                vf[mm][t] = *reinterpret_cast<const bf16x8*>(&sVt[t][cur][c * kKLd + 16 * mm + 8 * h2]);
            }
            if constexpr (P1) {
              const bf16x8 x[2] = {vf[mm][0], vf[mm][1]};
              mfma_h3s(x, ps3, ph3, pl3, o);
            } else {
              o = mfma_split<NP>(vf[mm], pf, o);
            }
          }
        }
      }
      if (kb + 1 < nkb) {
        sstore(cur ^ 1, std::integral_constant<int, 1 - S>{});
        if (vp) sstore3(cur ^ 1, std::integral_constant<int, 1 - S>{});
      }
      __syncthreads();
    };
#pragma unroll 1
    for (int kb = 0; kb < nkb; kb += 2) {
      block(kb, I0{});
      if (kb + 1 < nkb) block(kb + 1, I1{});
    }
  }
  if constexpr (MODE == 3) {
    if (!live || i >= L) return;
    const float inv = 1.f / (l + __shfl_xor(l, 32, 64));
    // z[i][c] = O^T[c][i] * y[i][c]: rows c = (r & 3) + 8 (r >> 2) + 4 h2 of each fragment
    // (y / z: bf16 in the bf16 mode, f32 in f16x3)
    const T* yrow = reinterpret_cast<const T*>(a.y) + (long)(r0 + i) * a.ldy;
    T* zrow = reinterpret_cast<T*>(a.z) + (long)(r0 + i) * a.hid;
#pragma unroll
    for (int f = 0; f < NF; ++f)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = fz * NF * 32 + f * 32 + 8 * g + 4 * h2;
        if (c0 < a.hid) {
          float ov[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            ov[e] = o3[f][4 * g + e] * inv;  // (P1: o3 and l both carry 2^11)
          if constexpr (SPLIT) {
            const float4 yv = *reinterpret_cast<const float4*>(yrow + c0);
            *reinterpret_cast<float4*>(zrow + c0) =
                make_float4(ov[0] * yv.x, ov[1] * yv.y, ov[2] * yv.z, ov[3] * yv.w);
          } else {
            const bf16x4 yv = *reinterpret_cast<const bf16x4*>(yrow + c0);
            bf16x4 zv;
#pragma unroll
            for (int e = 0; e < 4; ++e) zv[e] = (__bf16)(ov[e] * (float)yv[e]);
            *reinterpret_cast<bf16x4*>(zrow + c0) = zv;
          }
        }
      }
  }
  if constexpr (MODE == 1 || MODE == 2) {
    if (!live || i >= L) return;
    float inv = 1.f;
    if constexpr (MODE == 1) {
      const float lt = l + __shfl_xor(l, 32, 64);
      inv = 1.f / lt;  // (P1: o and lt both carry 2^11)
      if (h2 == 0) a.stats_out[(long)(r0 + i) * H + h] = m + __log2f(lt) - kE;
    } else if constexpr (P1) {
      inv = 1.f / 2048.f;  // mode 2: o carries 2^11
    }
    // O^T rows = value dims d = (r&3) + 8 (r>>2) + 4 h2; d < 12 valid
    T* dst = reinterpret_cast<T*>(a.out) + (long)(r0 + i) * ldv + 12 * h;
    if constexpr (SPLIT) {
      const float4 v0 = make_float4(o[0] * inv, o[1] * inv, o[2] * inv, o[3] * inv);
      const float4 v1 = make_float4(o[4] * inv, o[5] * inv, o[6] * inv, o[7] * inv);
      *reinterpret_cast<float4*>(dst + 4 * h2) = v0;
      if (h2 == 0) *reinterpret_cast<float4*>(dst + 8) = v1;
    } else {
      bf16x4 v0, v1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] = (__bf16)(o[e] * inv);
        v1[e] = (__bf16)(o[4 + e] * inv);
      }
      *reinterpret_cast<bf16x4*>(dst + 4 * h2) = v0;  // d 0..3 (h2 = 0) / 4..7 (h2 = 1)
      if (h2 == 0) *reinterpret_cast<bf16x4*>(dst + 8) = v1;  // d 8..11
    }
  }
}

// gfx950: one workgroup may hold all 160 KiB of a CU's LDS, static + dynamic together
constexpr size_t kLdsPerCu = 160 * 1024;

// the static LDS of a kernel instantiation (hipFuncGetAttributes, memoised per function)
static size_t kernel_static_lds(const void* fn) {
  static std::mutex mu;
  static std::unordered_map<const void*, size_t> memo;
  std::lock_guard<std::mutex> g(mu);
  auto it = memo.find(fn);
  if (it != memo.end()) return it->second;
  hipFuncAttributes at{};
  ZASR_HIP_CHECK(hipFuncGetAttributes(&at, fn));
  return memo[fn] = at.sharedSizeBytes;
}

// launch one flash-attention instantiation: its positional stage (dynamic LDS) must fit beside
// the template's static key / value staging, and a failed launch must not leave the output
// holding stale workspace data (checked right after the launch)
template <int MODE, int NP, int FMT, int NF>
static void launch_flash_one(const AttnFlashArgs& a, dim3 grid, size_t lds, hipStream_t st) {
  const void* fn = reinterpret_cast<const void*>(&attn_flash_kernel<MODE, NP, FMT, NF>);
  const size_t stat = kernel_static_lds(fn);
  if (lds + stat > kLdsPerCu)
    throw std::runtime_error("attention: sequence of " + std::to_string(a.max_len) +
                             " frames needs " + std::to_string(lds + stat) +
                             " B of LDS (positional stage + static staging), over the " +
                             std::to_string(kLdsPerCu) + " B of a gfx950 CU");
  ZASR_LAUNCH((attn_flash_kernel<MODE, NP, FMT, NF>), grid, dim3(256), lds, st, a);
}

template <int NP, int FMT = 0>
void launch_flash_np(const AttnFlashArgs& a, int mode, size_t lds, hipStream_t st) {
  const dim3 grid(cdiv(a.max_len, 128), a.nseq, mode == 0 ? 1 : a.H);
  if (mode == 0)
    launch_flash_one<0, NP, FMT, 1>(a, grid, lds, st);
  else if (mode == 1)
    launch_flash_one<1, NP, FMT, 1>(a, grid, lds, st);
  else
    launch_flash_one<2, NP, FMT, 1>(a, grid, lds, st);
}

void launch_attn_flash(const AttnFlashArgs& a, int mode, hipStream_t st) {
  if (a.nseq <= 0 || a.max_len <= 0) return;
  if (mode == 3) {
    ZASR_REQUIRE((a.pieces == 1 || a.pieces == kPiecesF16) && a.t1t && a.o8 && a.y && a.z &&
                     a.hid > 0 && a.hid % 4 == 0 && a.ldt % 8 == 0 && a.ldy % 4 == 0,
                 "attention mode 3: the bf16 or f16x3 mode, hid % 4 == 0");
    const size_t lds = (size_t)(a.max_len + kPosPad) * sizeof(float4);
    // 5 fragments for hid = 144 (one chunk) and 288 (two), 6 for 192 (one) and 384 (two)
    const int nft = cdiv(a.hid, 32);
    if (a.pieces == kPiecesF16) {  // f16x3: two accumulators and two V^T images per fragment
      // 3 value fragments per block (2 measured 4.87 vs 4.08 ms per hour)
      const dim3 grid(cdiv(a.max_len, 128), a.nseq, cdiv(nft, 3));
      launch_flash_one<3, 2, 1, 3>(a, grid, lds, st);
      return;
    }
    // (one pass, online: 5-6 fragments at one wave per SIMD beat 4 fragments at two, 1.63 vs
    // 2.08 ms per hour; the two-pass form took 2.02)
    const int nf = (nft % 5 == 0 || nft == 9) ? 5 : 6;
    const dim3 grid(cdiv(a.max_len, 128), a.nseq, cdiv(nft, nf));
    if (nf == 5)
      launch_flash_one<3, 1, 0, 5>(a, grid, lds, st);
    else
      launch_flash_one<3, 1, 0, 6>(a, grid, lds, st);
    return;
  }
  ZASR_REQUIRE(a.H % 2 == 0, "attention: the bf16 kernels need an even head count (16-byte q/k rows)");
  const size_t lds = (size_t)(a.max_len + kPosPad) * sizeof(float4);
  if (a.pieces == 1)
    launch_flash_np<1>(a, mode, lds, st);
  else if (a.pieces == 2)
    launch_flash_np<2>(a, mode, lds, st);
  else if (a.pieces == 3)
    launch_flash_np<3>(a, mode, lds, st);
  else if (a.pieces == kPiecesF16)
    launch_flash_np<2, 1>(a, mode, lds, st);
  else
    throw std::runtime_error("attention: pieces must be 1, 2, 3 or kPiecesF16");
}

// =====================================================================================
// t1^T = (tanh(s) * x)^T in bf16: h3 [R][3 hid] f32 -> t1t [hid][R8].  Tile 64 rows x 64
// channels transposed through LDS; packed row r of sequence b goes to column
// r + (o32_b - off_b); the last row of a sequence also writes the zero padding up to
// o32_b + L32_b (the K padding of the split modes' z-sliced gemm_x3).
// =====================================================================================
__device__ __forceinline__ float4 h3_load4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 h3_load4(const __bf16* p) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return make_float4((float)v[0], (float)v[1], (float)v[2], (float)v[3]);
}

// NP > 1 (split modes): NP bf16 pieces of t1 per element, piece t at t1t + t * hid * R8;
// NP = kPiecesF16: the two fp16 pieces hi, (t1 - hi) * 2^11 (gemm_dev.h split_h8)
template <typename TH, int NP>
__global__ __launch_bounds__(256) void nonlin_prep_t_kernel(const TH* __restrict__ h3,
                                                            const int* __restrict__ off,
                                                            const int* __restrict__ o8,
                                                            const int* __restrict__ map, int R,
                                                            int hid, int R8,
                                                            __bf16* __restrict__ t1t) {
  // tiled over the OUTPUT: 64 columns of t1t (packed rows of one or two sequences, or their
  // zero padding up to L32) x 64 channels, so every store is a 32-byte piece of a channel's
  // contiguous column run and the padding needs no separate pass
  __shared__ float tile[64][65];
  __shared__ int sRow[64];
  const int col0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  if (tid < 64) {
    const int col = col0 + tid;
    int lo = 0, hi = map[R - 1];  // (trailing empty sequences own no columns)  // the sequence owning column col: largest b with o8[b] <= col
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (o8[mid] <= col) lo = mid;
      else hi = mid - 1;
    }
    const int j = col - o8[lo];
    sRow[tid] = (col < R8 && j < off[lo + 1] - off[lo]) ? off[lo] + j : -1;
  }
  __syncthreads();
  float4 sv[4], xv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + 256 * k;
    const int rl = idx >> 4, c4 = idx & 15;
    const int r = sRow[rl];
    const int cc = c0 + 4 * c4 < hid ? c0 + 4 * c4 : hid - 4;
    const TH* row = h3 + (long)(r < 0 ? 0 : r) * 3 * hid;
    sv[k] = h3_load4(row + cc);
    xv[k] = h3_load4(row + hid + cc);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int idx = tid + 256 * k;
    const int rl = idx >> 4, c4 = idx & 15;
    const float m = sRow[rl] < 0 ? 0.f : 1.f;  // padding columns: zeros
    tile[4 * c4 + 0][rl] = tanhf(sv[k].x) * xv[k].x * m;
    tile[4 * c4 + 1][rl] = tanhf(sv[k].y) * xv[k].y * m;
    tile[4 * c4 + 2][rl] = tanhf(sv[k].z) * xv[k].z * m;
    tile[4 * c4 + 3][rl] = tanhf(sv[k].w) * xv[k].w * m;
  }
  __syncthreads();
  // channel cl, columns 16 g .. 16 g + 15: reads tile row cl (stride 65: conflict-free)
  const int cl = tid >> 2, g = tid & 3;
  const int ch = c0 + cl;
  const int cs = col0 + 16 * g;
  if (ch >= hid || cs >= R8) return;  // R8 % 32 == 0: a 16-column group is all in or all out
  float v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = tile[cl][16 * g + i];
  typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
  __bf16* dst = t1t + (long)ch * R8 + cs;
  if constexpr (NP == kPiecesF16) {
    typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));
    f16x8_t h[2], l[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const _Float16 hh = (_Float16)v[i];
      h[i >> 3][i & 7] = hh;
      l[i >> 3][i & 7] = (_Float16)((v[i] - (float)hh) * kF16Lo);
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      *reinterpret_cast<f16x8_t*>(dst + 8 * q) = h[q];
      *reinterpret_cast<f16x8_t*>(dst + (long)hid * R8 + 8 * q) = l[q];
    }
  } else {
#pragma unroll
    for (int t = 0; t < NP; ++t) {
      bf16x8_t p[2];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const __bf16 hh = (__bf16)v[i];
        p[i >> 3][i & 7] = hh;
        if (t + 1 < NP) v[i] -= (float)hh;
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) *reinterpret_cast<bf16x8_t*>(dst + (long)t * hid * R8 + 8 * q) = p[q];
    }
  }
}

void launch_nonlin_prep_t(const void* h3, bool h3_bf16, const int* off, const int* o8,
                          const int* map, int R, int hid, int R8, void* t1t, hipStream_t st,
                          int pieces) {
  if (R <= 0) return;
  ZASR_REQUIRE(hid % 4 == 0, "nonlin_prep_t: hid must be a multiple of 4");
  ZASR_REQUIRE(pieces == 1 || (!h3_bf16 && (pieces == 2 || pieces == 3 || pieces == kPiecesF16)),
               "nonlin_prep_t: pieces must be 1 (or 2 / 3 / kPiecesF16 for an f32 h3)");
  ZASR_REQUIRE(R8 % 32 == 0, "nonlin_prep_t: t1t columns are 32-padded per sequence");
  const dim3 grid(cdiv(R8, 64), cdiv(hid, 64));
  __bf16* out = reinterpret_cast<__bf16*>(t1t);
  const float* h3f = reinterpret_cast<const float*>(h3);
  if (h3_bf16)
    ZASR_LAUNCH((nonlin_prep_t_kernel<__bf16, 1>), grid, dim3(256), 0, st,
                       reinterpret_cast<const __bf16*>(h3), off, o8, map, R, hid, R8, out);
  else if (pieces == 1)
    ZASR_LAUNCH((nonlin_prep_t_kernel<float, 1>), grid, dim3(256), 0, st, h3f, off, o8,
                       map, R, hid, R8, out);
  else if (pieces == 2)
    ZASR_LAUNCH((nonlin_prep_t_kernel<float, 2>), grid, dim3(256), 0, st, h3f, off, o8,
                       map, R, hid, R8, out);
  else if (pieces == kPiecesF16)
    ZASR_LAUNCH((nonlin_prep_t_kernel<float, kPiecesF16>), grid, dim3(256), 0, st, h3f,
                       off, o8, map, R, hid, R8, out);
  else
    ZASR_LAUNCH((nonlin_prep_t_kernel<float, 3>), grid, dim3(256), 0, st, h3f, off, o8,
                       map, R, hid, R8, out);
}

}  // namespace zasr
