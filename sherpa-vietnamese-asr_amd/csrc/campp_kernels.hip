// CAM++ speaker-embedding kernels (the model is the reference's
// convert_onnx/export_campplus_onnx.py:17-270 CAMPPlus, eval mode, BatchNorm folded into the
// adjacent convolution where no nonlinearity separates them).  The dense projections (TDNN,
// dense-block 1x1 / k3 convs, transit and output layers) run on the exact-f32 MFMA GEMM
// (gemm.hip) with im2col operands; the kernels here are the FCM head's 2-D convolutions, the
// BN-ReLU pre-activations, the CAM context masks, statistics pooling and the fbank CMVN.
//
// Layouts: head [N][C][F][T] (NCHW, H = frequency, W = time); TDNN part channels-last
// [N * T2][C] so every 1 x 1 convolution is a plain GEMM.
#include "common.h"
#include "kernels.h"

namespace zasr {

// ---------------------------------------------------------------------------------------
// FCM 2-D convolution, 32 output channels, kernel KS x KS (3: pad 1, 1: pad 0), stride
// (sf, 1).  Block = 4 waves x 64 lanes: lane = time position of a 64-frame tile, wave w =
// output channels 8w .. 8w + 7 (weights read wave-uniformly from LDS: broadcast).  The input
// rows the tile needs (Ci x KS x 66 frames) are staged in LDS.
// Epilogue: y = acc * scale[co] + shift[co] (+ res) then ReLU (flags); output either NCHW or
// (tdnn_out) the TDNN layout [N][T][Co * Fo] with channel co * Fo + fo.
// ---------------------------------------------------------------------------------------
template <int KS, int CIMAX>
__global__ __launch_bounds__(256) void campp_conv2d_kernel(CamppConv2d a) {
  constexpr int CO = 32, TT = 64, PAD = KS / 2, TW = TT + KS - 1;
  // LDS sized for CIMAX input channels: the FCM head's first convolution (Ci = 1) stages
  // 2 KB instead of 61 KB, so 8 blocks (not 2) share a CU
  __shared__ float sW[CO * CIMAX * KS * KS];
  __shared__ float sX[CIMAX * KS * TW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int t0 = blockIdx.x * TT, fo = blockIdx.y, n = blockIdx.z;
  const int Ci = a.ci;
  const int nw = CO * Ci * KS * KS;
  for (int i = tid; i < nw; i += 256) sW[i] = a.w[i];
  for (int i = tid; i < Ci * KS * TW; i += 256) {
    const int ci = i / (KS * TW), r = (i / TW) % KS, tt = i % TW;
    const int f = fo * a.sf + r - PAD, t = t0 + tt - PAD;
    float v = 0.f;
    if (f >= 0 && f < a.fi && t >= 0 && t < a.T)
      v = a.in_tf ? a.x[((long)n * a.T + t) * a.fi + f]  // fbank features [n][T][F] (ci = 1)
                  : a.x[(((long)n * Ci + ci) * a.fi + f) * a.T + t];
    sX[i] = v;
  }
  __syncthreads();
  const int t = t0 + lane;
  float acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = 0.f;
  for (int ci = 0; ci < Ci; ++ci) {
#pragma unroll
    for (int r = 0; r < KS; ++r)
#pragma unroll
      for (int q = 0; q < KS; ++q) {
        const float x = sX[(ci * KS + r) * TW + lane + q];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = fmaf(x, sW[((w * 8 + c) * Ci + ci) * KS * KS + r * KS + q], acc[c]);
      }
  }
  if (t >= a.T) return;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const int co = w * 8 + c;
    float y = fmaf(acc[c], a.scale[co], a.shift[co]);
    const long o = (((long)n * CO + co) * a.fo + fo) * a.T + t;
    if (a.res) y += a.res[o];
    if (a.relu) y = fmaxf(y, 0.f);
    if (a.tdnn_out)
      a.y[((long)n * a.T + t) * (CO * a.fo) + co * a.fo + fo] = y;
    else
      a.y[o] = y;
  }
}

// ---------------------------------------------------------------------------------------
// The same convolution for Ci = 32 as an implicit GEMM on the exact-f32 MFMA
// (v_mfma_f32_16x16x4f32): O^T[co][pos] = sum_k W[co][k] X^T[k][pos], k = (r KS + q) Ci + ci.
// A block owns `rb` consecutive output frequency rows of one window and slides down them two
// rows at a time: 4 waves = 2 rows x 2 halves of T (<= 160, 5 tiles of 16 positions each),
// 2 co tiles of 16.  All weights are staged in LDS once per block (pre-permuted on the host);
// the input lives in a ring of ROWS = sf + KS rows (slot = (f + pad) mod ROWS) and the 2 sf
// rows the next step needs are loaded into registers before the MFMA loop and written into the
// slots just retired after it, so HBM traffic overlaps the matrix work.  Channel planes are TW
// floats apart with ROWS * TW = 16 mod 32 and the weight rows XOR-swizzled by k parity, so
// both halves of each ds_read_b32 are bank-conflict-free.  Epilogue as campp_conv2d_kernel.
// ---------------------------------------------------------------------------------------
namespace {
constexpr int cx_tw(int rows) {  // smallest TW >= 162 with rows * TW = 16 (mod 32)
  int tw = 162;
  while ((rows * tw) % 32 != 16) ++tw;
  return tw;
}
constexpr int kCxCols = 162;  // staged columns: positions < 160 read columns < 162

__device__ inline void cx_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// Input staging is per wave and per plane-row (channel ci of input row g, kCxCols columns
// from t = -pad): wave w takes plane-rows p = w + 4 i (rr = p / 32, ci = p % 32), so the row
// and LDS addresses are scalar and a lane only adds its columns lane + 64 c (c < 3).  Loads go
// through a buffer descriptor over this window's [32][fi][T] planes: padding and rows outside
// [0, fi) get an out-of-range offset and load 0, so the loads are unconditional.
struct CxLane {
  int lt[3];  // t of column lane + 64 c, or -1 when it is padding
};
__device__ inline CxLane cx_lane(int lane, int pad, int T) {
  CxLane l;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int col = lane + 64 * c, t = col - pad;
    l.lt[c] = (col < kCxCols && t >= 0 && t < T) ? t : -1;
  }
  return l;
}
__device__ inline void cx_load_prow(__amdgpu_buffer_rsrc_t rs, const CamppConv2d& a, int g, int ci,
                                    const CxLane& l, float (&v)[3]) {
  const bool rowok = g >= 0 && g < a.fi;
  const int base = (ci * a.fi + g) * a.T;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const int off = (rowok && l.lt[c] >= 0) ? (base + l.lt[c]) * 4 : (int)0x80000000;
    v[c] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
  }
}
template <int ROWS, int TW, int PAD>
__device__ inline void cx_store_prow(float* sX, int g, int ci, int lane, const float (&v)[3]) {
  float* d = sX + (ci * ROWS + (g + PAD) % ROWS) * TW + lane;
  d[0] = v[0];
  d[64] = v[1];
  if (lane + 128 < kCxCols) d[128] = v[2];
}
}  // namespace

template <int KS, int SF, bool RES>
__global__ __launch_bounds__(256, 1) void campp_conv2d_mfma_kernel(CamppConv2d a, int rb) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int CI = 32, PAD = KS / 2, ROWS = SF + KS, NEW = 2 * SF, TW = cx_tw(ROWS);
  constexpr int K = KS * KS * CI, NT = 5;  // NT position tiles of 16 per wave
  __shared__ float sX[CI * ROWS * TW];
  __shared__ float sW[K * 32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = blockIdx.y, fo_begin = blockIdx.x * rb, fo_end = min(a.fo, fo_begin + rb);
  const int T = a.T;
  // weights arrive pre-permuted (a.wk: the sW image, k-major, XOR-swizzled): a float4 copy
  {
    const float4* src = reinterpret_cast<const float4*>(a.wk);
    float4* dst = reinterpret_cast<float4*>(sW);
    constexpr int NW4 = K * 32 / 4, NI = (NW4 + 255) / 256;
    float4 v[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = tid + 256 * i;
      v[i] = src[e < NW4 ? e : NW4 - 1];
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int e = tid + 256 * i;
      if (e < NW4) dst[e] = v[i];
    }
  }
  // buffer descriptor over this window's input planes
  const float* xw = a.x + (long)n * CI * a.fi * T;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(unsigned long)xw);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((unsigned long)xw >> 32));
  const int nbytes = __builtin_amdgcn_readfirstlane(CI * a.fi * T * 4);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(((unsigned long)hi << 32) | lo), 0, nbytes, 0x00020000);
  const CxLane cl = cx_lane(lane, PAD, T);
  // the first ROWS input rows, 4 plane-rows (12 loads) in flight per wave
  {
    const int g0 = fo_begin * SF - PAD;
#pragma unroll 1
    for (int i0 = 0; i0 < ROWS * 8; i0 += 4) {
      float v[4][3];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = w + 4 * (i0 + u);
        cx_load_prow(rs, a, g0 + (p >> 5), p & 31, cl, v[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int p = w + 4 * (i0 + u);
        cx_store_prow<ROWS, TW, PAD>(sX, g0 + (p >> 5), p & 31, lane, v[u]);
      }
    }
  }
  __syncthreads();
  const int orow = w >> 1, tile0 = 5 * (w & 1);
  const int r16 = lane & 15, g4 = lane >> 4;
  const int wsw = 16 * (g4 & 1);  // k parity of this lane
  // epilogue constants of this lane's channels 16 m + 4 g4 + e
  float esc[2][4], esh[2][4];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      esc[m][e] = a.scale[16 * m + 4 * g4 + e];
      esh[m][e] = a.shift[16 * m + 4 * g4 + e];
    }
  for (int fo = fo_begin; fo < fo_end; fo += 2) {
    const int fw = fo + orow;
    // the residual this step's outputs add, loaded with the rows (clamped, unconditional)
    float rv[RES ? 2 : 1][RES ? NT : 1][4];
    if constexpr (RES) {
      const int fr = min(fw, a.fo - 1);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int t = min(16 * (tile0 + u) + r16, T - 1);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            rv[m][u][e] = a.res[(((long)n * 32 + 16 * m + 4 * g4 + e) * a.fo + fr) * T + t];
      }
    }
    // prefetch the rows the next step adds (rows past fi load as 0)
    const int gn = fo * SF - PAD + ROWS;
    float pv[NEW * 8][3];
#pragma unroll
    for (int i = 0; i < NEW * 8; ++i) {
      const int p = w + 4 * i;
      cx_load_prow(rs, a, gn + (p >> 5), p & 31, cl, pv[i]);
    }
    f32x4 acc[2][NT];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int u = 0; u < NT; ++u) acc[m][u] = f32x4{0.f, 0.f, 0.f, 0.f};
    // K loop flattened to NS = KS KS CI / 4 steps, operands double-buffered in registers so
    // step s + 1's LDS reads are in flight under step s's 10 MFMAs
    const float* xrow[KS];
#pragma unroll
    for (int r = 0; r < KS; ++r)
      xrow[r] = sX + ((fw * SF + r) % ROWS) * TW + tile0 * 16 + r16;  // input row fw sf - pad + r
    constexpr int NS = KS * KS * CI / 4;
    float opA[2][2], opB[2][NT];
    auto ld = [&](int st, float (&A)[2], float (&B)[NT]) {
      const int rq = st / (CI / 4), j = st % (CI / 4), r = rq / KS, q = rq % KS;
      const int ci = 4 * j + g4, k = rq * CI + ci;
      A[0] = sW[k * 32 + (r16 ^ wsw)];
      A[1] = sW[k * 32 + ((16 + r16) ^ wsw)];
      const float* xc = xrow[r] + q + ci * ROWS * TW;
#pragma unroll
      for (int u = 0; u < NT; ++u) B[u] = xc[16 * u];
    };
    ld(0, opA[0], opB[0]);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const int cb = st & 1;
      if (st + 1 < NS) ld(st + 1, opA[cb ^ 1], opB[cb ^ 1]);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        acc[0][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(opA[cb][0], opB[cb][u], acc[0][u], 0, 0, 0);
        acc[1][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(opA[cb][1], opB[cb][u], acc[1][u], 0, 0, 0);
      }
    }
    // every wave is done with the retiring slots: fill them with the prefetched rows
    cx_lds_barrier();
#pragma unroll
    for (int i = 0; i < NEW * 8; ++i) {
      const int p = w + 4 * i;
      cx_store_prow<ROWS, TW, PAD>(sX, gn + (p >> 5), p & 31, lane, pv[i]);
    }
    // epilogue: lane holds positions t = 16 (tile0 + u) + r16, channels 16 m + 4 g4 + e
    if (fw < fo_end) {
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int t = 16 * (tile0 + u) + r16;
        if (t >= T) continue;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int co = 16 * m + 4 * g4 + e;
            float y = fmaf(acc[m][u][e], esc[m][e], esh[m][e]);
            const long o = (((long)n * 32 + co) * a.fo + fw) * T + t;
            if constexpr (RES) y += rv[m][u][e];
            if (a.relu) y = fmaxf(y, 0.f);
            if (a.tdnn_out)
              a.y[((long)n * T + t) * (32 * a.fo) + co * a.fo + fw] = y;
            else
              a.y[o] = y;
          }
      }
    }
    // the ring slots written above must be complete before the next step reads them; the
    // output stores need not (an LDS-only barrier leaves them in flight)
    cx_lds_barrier();
  }
}

// the MFMA kernel's weight image: w [32][32][ks][ks] -> [k = (r ks + q) 32 + ci][co ^ 16 (k & 1)]
void campp_conv2d_permute_weights(const float* w, int ks, float* out) {
  const int K = ks * ks * 32;
  for (int co = 0; co < 32; ++co)
    for (int ci = 0; ci < 32; ++ci)
      for (int rq = 0; rq < ks * ks; ++rq) {
        const int k = rq * 32 + ci;
        out[k * 32 + (co ^ (16 * (k & 1)))] = w[(co * 32 + ci) * ks * ks + rq];
      }
  (void)K;
}

void launch_campp_conv2d(const CamppConv2d& a, int ks, hipStream_t st) {
  ZASR_REQUIRE(a.ci <= 32 && (ks == 1 || ks == 3), "campp conv2d: Ci <= 32, kernel 1 or 3");
  // the 3 x 3 convolutions take the MFMA kernel; the 1 x 1 shortcut (a quarter of the
  // rows' work, no reuse across taps) stays on the direct kernel, which measured faster
  if (ks == 3 && a.wk && a.ci == 32 && !a.in_tf && a.T <= 160 &&
      (a.sf == 1 || a.sf == 2)) {
    // rows per block: about 2048 blocks per launch, an even row count, at least 2
    const int pairs = cdiv(a.fo, 2);
    const int chunks = std::max(1, std::min(pairs, cdiv(2048, a.n)));
    const int rb = 2 * cdiv(pairs, chunks);
    const dim3 grid(cdiv(a.fo, rb), a.n);
#define ZASR_CX(KSV, SFV, RESV) \
  ZASR_LAUNCH((campp_conv2d_mfma_kernel<KSV, SFV, RESV>), grid, dim3(256), 0, st, a, rb)
    if (a.sf == 1 && a.res) ZASR_CX(3, 1, true);
    else if (a.sf == 1) ZASR_CX(3, 1, false);
    else if (a.res) ZASR_CX(3, 2, true);
    else ZASR_CX(3, 2, false);
#undef ZASR_CX
    return;
  }
  dim3 grid(cdiv(a.T, 64), a.fo, a.n);
  if (ks == 3 && a.ci == 1) ZASR_LAUNCH((campp_conv2d_kernel<3, 1>), grid, dim3(256), 0, st, a);
  else if (ks == 3) ZASR_LAUNCH((campp_conv2d_kernel<3, 32>), grid, dim3(256), 0, st, a);
  else ZASR_LAUNCH((campp_conv2d_kernel<1, 32>), grid, dim3(256), 0, st, a);
}

// y[r][c] = relu(x[r][c] * s[c] + b[c]), c < C (x row stride ldx, y row stride C)
__global__ void campp_bnrelu_kernel(const float* __restrict__ x, int ldx, long R, int C,
                                    const float* __restrict__ s, const float* __restrict__ b,
                                    float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4n = C / 4;
  if (i >= R * c4n) return;
  const long r = i / c4n;
  const int c = (int)(i - r * c4n) * 4;
  const float4 v = *reinterpret_cast<const float4*>(x + r * ldx + c);
  const float4 sv = *reinterpret_cast<const float4*>(s + c), bv = *reinterpret_cast<const float4*>(b + c);
  *reinterpret_cast<float4*>(y + r * C + c) =
      make_float4(fmaxf(fmaf(v.x, sv.x, bv.x), 0.f), fmaxf(fmaf(v.y, sv.y, bv.y), 0.f),
                  fmaxf(fmaf(v.z, sv.z, bv.z), 0.f), fmaxf(fmaf(v.w, sv.w, bv.w), 0.f));
}

void launch_campp_bnrelu(const float* x, int ldx, long R, int C, const float* s, const float* b,
                         float* y, hipStream_t st) {
  ZASR_REQUIRE(C % 4 == 0 && ldx % 4 == 0, "campp bnrelu: channels must be multiples of 4");
  const long n = R * (C / 4);
  if (n <= 0) return;
  ZASR_LAUNCH(campp_bnrelu_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st, x, ldx,
                     R, C, s, b, y);
}

// im2col of a 1-D convolution over sequences of Tin frames (channels-last, row stride ldx):
// out[n * Tout + t][k * C + c] = x[n * Tin + t * stride + k * dil - pad][c] (0 outside)
__global__ void campp_im2col1d_kernel(const float* __restrict__ x, int ldx, int N, int Tin,
                                      int Tout, int C, int K, int stride, int dil, int pad,
                                      float* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int c4n = C / 4;
  const long total = (long)N * Tout * K * c4n;
  if (i >= total) return;
  const int c = (int)(i % c4n) * 4;
  const long j = i / c4n;
  const int k = (int)(j % K);
  const long r = j / K;
  const int n = (int)(r / Tout), t = (int)(r - (long)n * Tout);
  const int ts = t * stride + k * dil - pad;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ts >= 0 && ts < Tin) v = *reinterpret_cast<const float4*>(x + ((long)n * Tin + ts) * ldx + c);
  *reinterpret_cast<float4*>(out + r * ((long)K * C) + k * C + c) = v;
}

void launch_campp_im2col1d(const float* x, int ldx, int N, int Tin, int Tout, int C, int K,
                           int stride, int dil, int pad, float* out, hipStream_t st) {
  ZASR_REQUIRE(C % 4 == 0 && ldx % 4 == 0, "campp im2col: channels must be multiples of 4");
  const long n = (long)N * Tout * K * (C / 4);
  if (n <= 0) return;
  ZASR_LAUNCH(campp_im2col1d_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st, x,
                     ldx, N, Tin, Tout, C, K, stride, dil, pad, out);
}

// CAM context mask (CAMLayer.forward: context = mean_t(x) + seg_pooling(x); m = sigmoid(
// linear2(relu(linear1(context))))), block per (sequence n, segment g): 128 input channels
// (one per thread), the per-segment mask expanded to every frame of the segment:
// mexp[n * T + t][o] for t in segment g.  avg_pool1d(ceil_mode) divides a clipped last
// segment by its true length.
__global__ __launch_bounds__(256) void campp_cam_mask_kernel(CamppCamMask a) {
  __shared__ double sPart[2][2][128];
  __shared__ float sCtx[128];
  __shared__ float sZ[64];
  __shared__ float sM[32];
  const int tid = threadIdx.x, n = blockIdx.y, g = blockIdx.x;
  const int T = a.T, L = a.seg_len;
  const int s0 = g * L, s1 = min(T, s0 + L);
  // frame sums: channel c = tid % 128, frames of parity h = tid / 128, 8 loads in flight
  {
    const int c = tid & 127, h = tid >> 7;
    const float* x = a.h + (long)n * T * 128 + c;
    double tot = 0.0, seg = 0.0;
    int t = h;
    for (; t + 14 < T; t += 16) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[(long)(t + 2 * u) * 128];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int tu = t + 2 * u;
        tot += v[u];
        if (tu >= s0 && tu < s1) seg += v[u];
      }
    }
    for (; t < T; t += 2) {
      const float v = x[(long)t * 128];
      tot += v;
      if (t >= s0 && t < s1) seg += v;
    }
    sPart[h][0][c] = tot;
    sPart[h][1][c] = seg;
  }
  __syncthreads();
  if (tid < 128)
    sCtx[tid] = (float)((sPart[0][0][tid] + sPart[1][0][tid]) / T) +
                (float)((sPart[0][1][tid] + sPart[1][1][tid]) / (s1 - s0));
  __syncthreads();
  // linear1 + ReLU: 4 lanes per output, 32 channels each
  {
    const int j = tid >> 2, q = tid & 3;
    const float4* w = reinterpret_cast<const float4*>(a.w1 + j * 128 + q * 32);
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 v = w[i];
      const float* cx = sCtx + q * 32 + 4 * i;
      z = fmaf(v.x, cx[0], z);
      z = fmaf(v.y, cx[1], z);
      z = fmaf(v.z, cx[2], z);
      z = fmaf(v.w, cx[3], z);
    }
    z += __shfl_xor(z, 1);
    z += __shfl_xor(z, 2);
    if (q == 0) sZ[j] = fmaxf(z + a.b1[j], 0.f);
  }
  __syncthreads();
  // linear2 + sigmoid: 8 lanes per output, 8 inputs each
  {
    const int o = tid >> 3, q = tid & 7;
    const float4* w = reinterpret_cast<const float4*>(a.w2 + o * 64 + q * 8);
    const float4 v0 = w[0], v1 = w[1];
    const float* zz = sZ + q * 8;
    float m = v0.x * zz[0];
    m = fmaf(v0.y, zz[1], m);
    m = fmaf(v0.z, zz[2], m);
    m = fmaf(v0.w, zz[3], m);
    m = fmaf(v1.x, zz[4], m);
    m = fmaf(v1.y, zz[5], m);
    m = fmaf(v1.z, zz[6], m);
    m = fmaf(v1.w, zz[7], m);
    m += __shfl_xor(m, 1);
    m += __shfl_xor(m, 2);
    m += __shfl_xor(m, 4);
    if (q == 0) sM[o] = 1.f / (1.f + expf(-(m + a.b2[o])));
  }
  __syncthreads();
  for (int i = tid; i < (s1 - s0) * 8; i += 256) {
    const int t = s0 + i / 8, o4 = i % 8;
    *reinterpret_cast<float4*>(a.mexp + ((long)n * T + t) * 32 + 4 * o4) =
        *reinterpret_cast<const float4*>(sM + 4 * o4);
  }
}

void launch_campp_cam_mask(const CamppCamMask& a, hipStream_t st) {
  const int nseg = cdiv(a.T, a.seg_len);
  ZASR_LAUNCH(campp_cam_mask_kernel, dim3(nseg, a.n), dim3(256), 0, st, a);
}

// statistics pooling over T frames of relu(bn(x)) (the out_nonlinear BN-ReLU folded in):
// out[n][c] = mean, out[n][C + c] = unbiased std (StatsPool, f64 accumulation)
__global__ void campp_stats_kernel(const float* __restrict__ x, int N, int T, int C,
                                   const float* __restrict__ s, const float* __restrict__ b,
                                   float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i - n * C;
  const float sc = s[c], sh = b[c];
  double sum = 0.0;
  for (int t = 0; t < T; ++t) sum += fmaxf(fmaf(x[((long)n * T + t) * C + c], sc, sh), 0.f);
  const double mean = sum / T;
  double ss = 0.0;
  for (int t = 0; t < T; ++t) {
    const double d = fmaxf(fmaf(x[((long)n * T + t) * C + c], sc, sh), 0.f) - mean;
    ss += d * d;
  }
  out[(long)n * 2 * C + c] = (float)mean;
  out[(long)n * 2 * C + C + c] = T > 1 ? (float)sqrt(ss / (T - 1)) : NAN;
}

void launch_campp_stats(const float* x, int N, int T, int C, const float* s, const float* b,
                        float* out, hipStream_t st) {
  if (N * C <= 0) return;
  ZASR_LAUNCH(campp_stats_kernel, dim3(cdiv(N * C, 128)), dim3(128), 0, st, x, N, T, C, s,
                     b, out);
}

// per-utterance CMVN of fbank features: x[f][m] -= mean_f x[f][m] (one block per sequence,
// one thread per mel bin)
// per-sequence mean removal over frames: 12 frame groups x 80 bins per block, f64 partial
// sums (8 loads in flight per thread) combined in LDS
__global__ __launch_bounds__(960) void campp_cmvn_kernel(float* __restrict__ x,
                                                         const int* __restrict__ fr_off) {
  constexpr int G = 12;
  __shared__ double part[G][80];
  __shared__ float mean_s[80];
  const int s = blockIdx.x, m = threadIdx.x % 80, g = threadIdx.x / 80;
  const int a = fr_off[s], e = fr_off[s + 1];
  if (e <= a) return;
  double sum = 0.0;
  int f = a + g;
  for (; f + 7 * G < e; f += 8 * G) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = x[(long)(f + u * G) * 80 + m];
#pragma unroll
    for (int u = 0; u < 8; ++u) sum += v[u];
  }
  for (; f < e; f += G) sum += x[(long)f * 80 + m];
  part[g][m] = sum;
  __syncthreads();
  if (g == 0) {
    double t = 0.0;
    for (int i = 0; i < G; ++i) t += part[i][m];
    mean_s[m] = (float)(t / (e - a));
  }
  __syncthreads();
  const float mean = mean_s[m];
  for (f = a + g; f < e; f += G) x[(long)f * 80 + m] -= mean;
}

void launch_campp_cmvn(float* x, const int* fr_off, int nseq, hipStream_t st) {
  if (nseq <= 0) return;
  ZASR_LAUNCH(campp_cmvn_kernel, dim3(nseq), dim3(960), 0, st, x, fr_off);
}

// one block per window: 20 float4 per frame, consecutive threads on consecutive float4 of
// the window (coalesced reads of the packed rows and writes of the window tensor)
__global__ __launch_bounds__(256) void campp_gather_kernel(const float4* __restrict__ rows,
                                                           const int* __restrict__ win_row,
                                                           const int* __restrict__ win_n, int wf,
                                                           float4* __restrict__ out) {
  const int w = blockIdx.x;
  const long r0 = win_row[w];
  const int n = win_n[w];
  float4* o = out + (long)w * wf * 20;
  for (int i = threadIdx.x; i < wf * 20; i += 256) {
    const int t = i / 20;
    o[i] = t < n ? rows[r0 * 20 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

void launch_campp_gather(const float* rows, const int* win_row, const int* win_n, int nwin,
                         int wf, float* out, hipStream_t st) {
  if (nwin <= 0) return;
  ZASR_LAUNCH(campp_gather_kernel, dim3(nwin), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(rows), win_row, win_n, wf,
                     reinterpret_cast<float4*>(out));
}

}  // namespace zasr
