// Transducer search on device: modified beam search (greedy = beam 1) with Aho-Corasick
// hotword biasing, restating core/asr_engine.py:1023-1153 and core/hotword_context.py.
//
// Per frame t (host loop):   decoder_prep -> decoder_proj GEMM -> joiner GEMM -> search_step
//
// search_step: one 256-thread block per stream.
//   1. per live hypothesis row (wave-parallel): max, second max, sum exp, entropy terms
//      (the reference's f32 numpy log-softmax :1096-1098 and _compute_token_entropy :1159)
//   2. candidates lp = ((logit - max) - log(sum)) + float(score_h)   (f32, :1098-1100)
//      global top-k over H*V: per-thread sorted lists -> per-wave merge -> block merge
//   3. thread 0 expands the k candidates in descending order: blank keeps the sequence,
//      non-blank appends (hotword delta after top-k, :1127-1131); duplicates of the full
//      token sequence (identified by (length, 64-bit rolling hash)) merge with an f64
//      log-add (:1133-1138); emissions append a node {token, frame, parent, token logp,
//      row stats} so the winning sequence is recovered at the end by backtracking.
#include "common.h"
#include "kernels.h"

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

// returns the f64 log-add; *f64 = 1 when the reference's result type is np.float64
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

// candidate order: larger value first, then smaller flat index
__device__ __forceinline__ bool better(float v1, int i1, float v2, int i2) {
  return v1 > v2 || (v1 == v2 && i1 < i2);
}

}  // namespace

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
  hipLaunchKernelGGL(search_init_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, s, S, Hmax);
}

// decoder: relu(Conv1d(D, D, k=2, groups=D/4, no bias)(E[y2], E[y1])) per slot
__global__ void decoder_prep_kernel(const int* __restrict__ y1, const int* __restrict__ y2,
                                    int rows, const float* __restrict__ emb,
                                    const float* __restrict__ conv_w, int D,
                                    float* __restrict__ out) {
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)rows * D) return;
  int r = (int)(e / D), c = (int)(e - (long)r * D);
  const float* ea = emb + (long)y2[r] * D + (c & ~3);  // tap 0: older token
  const float* eb = emb + (long)y1[r] * D + (c & ~3);  // tap 1: newer token
  const float* w = conv_w + (long)c * 8;                // [ci][tap]
  float acc = 0.f;
#pragma unroll
  for (int ci = 0; ci < 4; ++ci) {
    acc = fmaf(w[ci * 2 + 0], ea[ci], acc);
    acc = fmaf(w[ci * 2 + 1], eb[ci], acc);
  }
  out[e] = fmaxf(acc, 0.f);
}

void launch_decoder_prep(const SearchState& s, int rows, const float* emb, const float* conv_w,
                         int D, float* out, hipStream_t st) {
  long n = (long)rows * D;
  if (n <= 0) return;
  hipLaunchKernelGGL(decoder_prep_kernel, dim3(cdivl(n, 256)), dim3(256), 0, st, s.y1, s.y2,
                     rows, emb, conv_w, D, out);
}

template <int KB>
__global__ __launch_bounds__(256) void search_step_kernel(SearchState st, const float* logits,
                                                          int V, int Hmax, int beam, int t,
                                                          const int* enc_len, HotwordTables hw) {
  const int s = blockIdx.x;
  if (t >= enc_len[s]) return;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int base = s * Hmax;

  __shared__ float sMax[kMaxBeam], sLogSum[kMaxBeam], sScore[kMaxBeam];
  __shared__ double sScoreD[kMaxBeam];
  __shared__ int sScoreF[kMaxBeam];
  __shared__ float4 sStats[kMaxBeam];
  __shared__ float cV[4 * KB];
  __shared__ int cI[4 * KB];
  __shared__ int sN;

  if (tid == 0) sN = st.nh[s];
  __syncthreads();
  const int n = sN;
  const float* rows = logits + (long)base * V;

  // ---- 1. per-hypothesis row statistics ----
  for (int h = wid; h < n; h += 4) {
    const float* row = rows + (long)h * V;
    float m1 = -INFINITY, m2 = -INFINITY;
    for (int v = lane; v < V; v += 64) {
      float x = row[v];
      if (x > m1) {
        m2 = m1;
        m1 = x;
      } else if (x > m2) {
        m2 = x;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float a1 = __shfl_xor(m1, o, 64), a2 = __shfl_xor(m2, o, 64);
      float hi = fmaxf(m1, a1);
      float lo = fmaxf(fminf(m1, a1), fmaxf(m2, a2));
      m1 = hi;
      m2 = lo;
    }
    float se = 0.f;
    for (int v = lane; v < V; v += 64) se += expf(row[v] - m1);
    se = wave_sum(se);
    float ent = 0.f, s3 = 0.f;
    for (int v = lane; v < V; v += 64) {
      float p = expf(row[v] - m1) / se;
      ent += p * logf(p + 1e-30f);
      s3 += powf(p, 1.0f / 3.0f);
    }
    ent = wave_sum(ent);
    s3 = wave_sum(s3);
    if (lane == 0) {
      sMax[h] = m1;
      sLogSum[h] = logf(se);
      sScore[h] = (float)st.lp[base + h];
      sScoreD[h] = st.lp[base + h];
      sScoreF[h] = st.lpf[base + h];
      sStats[h] = make_float4(-ent, s3, 1.0f / se, expf(m2 - m1) / se);
    }
  }
  __syncthreads();

  // ---- 2. top-k over n * V candidates ----
  float tv[KB];
  int ti[KB];
#pragma unroll
  for (int q = 0; q < KB; ++q) {
    tv[q] = -INFINITY;
    ti[q] = 0x7fffffff;
  }
  const int total = n * V;
  for (int idx = tid; idx < total; idx += 256) {
    const int h = idx / V;
    const float x = rows[idx];
    const float lpv = (x - sMax[h]) - sLogSum[h];
    // reference: f32 `lp[i, :] += score` (Python float) or f64 add rounded (np.float64)
    const float val = sScoreF[h] ? (float)((double)lpv + sScoreD[h]) : lpv + sScore[h];
    if (!better(val, idx, tv[KB - 1], ti[KB - 1])) continue;
#pragma unroll
    for (int q = KB - 1; q >= 0; --q) {
      const bool gt_prev = (q > 0) ? better(val, idx, tv[q - 1], ti[q - 1]) : false;
      const bool gt_cur = better(val, idx, tv[q], ti[q]);
      if (gt_prev) {
        tv[q] = tv[q - 1];
        ti[q] = ti[q - 1];
      } else if (gt_cur) {
        tv[q] = val;
        ti[q] = idx;
      }
    }
  }
  // per-wave merge: KB rounds of wave argmax over the lanes' list heads
  for (int round = 0; round < KB; ++round) {
    float bv = tv[0];
    int bi = ti[0];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      float ov = __shfl_xor(bv, o, 64);
      int oi = __shfl_xor(bi, o, 64);
      if (better(ov, oi, bv, bi)) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      cV[wid * KB + round] = bv;
      cI[wid * KB + round] = bi;
    }
    if (ti[0] == bi && bi != 0x7fffffff) {  // pop the winner's head (indices are unique)
#pragma unroll
      for (int q = 0; q < KB - 1; ++q) {
        tv[q] = tv[q + 1];
        ti[q] = ti[q + 1];
      }
      tv[KB - 1] = -INFINITY;
      ti[KB - 1] = 0x7fffffff;
    }
  }
  __syncthreads();

  // ---- 3. expansion, hotwords, dedup (serial, <= beam candidates) ----
  if (tid == 0) {
    const int k = beam < total ? beam : total;
    int ptr[4] = {0, 0, 0, 0};
    // copy previous hypotheses (read before overwrite)
    double plp[kMaxBeam];
    unsigned long long phash[kMaxBeam];
    int plen[kMaxBeam], py1[kMaxBeam], py2[kMaxBeam], phw[kMaxBeam], pnode[kMaxBeam];
    for (int h = 0; h < n; ++h) {
      plp[h] = st.lp[base + h];
      py2[h] = st.y2[base + h];
      phash[h] = st.hash[base + h];
      plen[h] = st.len[base + h];
      py1[h] = st.y1[base + h];
      phw[h] = st.hw[base + h];
      pnode[h] = st.node[base + h];
    }
    int nn = 0;
    for (int c = 0; c < k; ++c) {
      // next best among the 4 wave lists
      int bw = -1;
      for (int w = 0; w < 4; ++w) {
        if (ptr[w] >= KB) continue;
        if (bw < 0 || better(cV[w * KB + ptr[w]], cI[w * KB + ptr[w]], cV[bw * KB + ptr[bw]],
                             cI[bw * KB + ptr[bw]]))
          bw = w;
      }
      const float val = cV[bw * KB + ptr[bw]];
      const int idx = cI[bw * KB + ptr[bw]];
      ++ptr[bw];
      if (idx == 0x7fffffff) break;
      const int hi = idx / V, tok = idx - hi * V;
      double score = (double)val;
      unsigned long long key;
      int klen, ny1, ny2, nhw, nnode = -1;
      double tok_lp = 0.0;
      if (tok == 0) {
        key = phash[hi];
        klen = plen[hi];
        ny1 = py1[hi];
        ny2 = py2[hi];
        nhw = phw[hi];
        nnode = pnode[hi];
      } else {
        tok_lp = (double)val - plp[hi];
        nhw = phw[hi];
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
        key = hash_push(phash[hi], tok);
        klen = plen[hi] + 1;
        ny2 = py1[hi];
        ny1 = tok;
      }
      int found = -1;
      for (int j = 0; j < nn; ++j)
        if (st.len[base + j] == klen && st.hash[base + j] == key) {
          found = j;
          break;
        }
      if (found >= 0) {
        int f64 = 0;
        st.lp[base + found] = log_add(st.lp[base + found], st.lpf[base + found], score, 0, &f64);
        st.lpf[base + found] = f64;
        continue;
      }
      if (tok != 0) {
        const int nid = st.node_count[s]++;
        const long g = (long)s * st.node_cap + nid;
        st.node_tok[g] = tok;
        st.node_frame[g] = t;
        st.node_parent[g] = pnode[hi];
        st.node_lp[g] = tok_lp;
        st.node_stats[g] = sStats[hi];
        nnode = nid;
      }
      st.lp[base + nn] = score;
      st.lpf[base + nn] = 0;
      st.hash[base + nn] = key;
      st.len[base + nn] = klen;
      st.y1[base + nn] = ny1;
      st.y2[base + nn] = ny2;
      st.hw[base + nn] = nhw;
      st.node[base + nn] = nnode;
      ++nn;
    }
    st.nh[s] = nn;
  }
}

void launch_search_step(const SearchState& s, const float* logits, int V, int S, int Hmax,
                        int beam, int t, const int* enc_len, const HotwordTables& hw,
                        hipStream_t st) {
  if (S <= 0) return;
  ZASR_REQUIRE(beam >= 1 && beam <= kMaxBeam && beam <= Hmax, "beam out of range");
  dim3 grid(S), block(256);
  if (beam == 1)
    hipLaunchKernelGGL(search_step_kernel<1>, grid, block, 0, st, s, logits, V, Hmax, beam, t,
                       enc_len, hw);
  else if (beam <= 4)
    hipLaunchKernelGGL(search_step_kernel<4>, grid, block, 0, st, s, logits, V, Hmax, beam, t,
                       enc_len, hw);
  else if (beam <= 8)
    hipLaunchKernelGGL(search_step_kernel<8>, grid, block, 0, st, s, logits, V, Hmax, beam, t,
                       enc_len, hw);
  else
    hipLaunchKernelGGL(search_step_kernel<16>, grid, block, 0, st, s, logits, V, Hmax, beam, t,
                       enc_len, hw);
}

// finalize (:1142-1148), length-normalised pick (:1151), backtrack the emission chain
__global__ void search_final_kernel(SearchState st, int S, int Hmax, HotwordTables hw,
                                    int out_cap, int* out_tok, int* out_frame, double* out_lp,
                                    float4* out_stats, int* out_count) {
  int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  const int base = s * Hmax;
  const int n = st.nh[s];
  int best = 0;
  double best_v = -INFINITY;
  for (int h = 0; h < n; ++h) {
    double lp = st.lp[base + h];
    if (hw.num_states > 0) lp += -hw.node_score[st.hw[base + h]];
    double v = lp / (double)(st.len[base + h] > 1 ? st.len[base + h] : 1);
    if (h == 0 || v > best_v) {
      best_v = v;
      best = h;
    }
  }
  int cnt = 0;
  for (int nd = st.node[base + best]; nd >= 0; nd = st.node_parent[(long)s * st.node_cap + nd])
    ++cnt;
  if (cnt > out_cap) cnt = out_cap;
  int pos = cnt - 1;
  for (int nd = st.node[base + best]; nd >= 0 && pos >= 0;
       nd = st.node_parent[(long)s * st.node_cap + nd], --pos) {
    const long g = (long)s * st.node_cap + nd;
    const long o = (long)s * out_cap + pos;
    out_tok[o] = st.node_tok[g];
    out_frame[o] = st.node_frame[g];
    out_lp[o] = st.node_lp[g];
    out_stats[o] = st.node_stats[g];
  }
  out_count[s] = cnt;
}

void launch_search_final(const SearchState& s, int S, int Hmax, const HotwordTables& hw,
                         int out_cap, int* out_tok, int* out_frame, double* out_lp,
                         float4* out_stats, int* out_count, hipStream_t st) {
  if (S <= 0) return;
  hipLaunchKernelGGL(search_final_kernel, dim3(cdiv(S, 64)), dim3(64), 0, st, s, S, Hmax, hw,
                     out_cap, out_tok, out_frame, out_lp, out_stats, out_count);
}

}  // namespace zasr
