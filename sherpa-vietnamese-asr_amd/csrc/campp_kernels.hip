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
template <int KS>
__global__ __launch_bounds__(256) void campp_conv2d_kernel(CamppConv2d a) {
  constexpr int CO = 32, TT = 64, PAD = KS / 2, TW = TT + KS - 1;
  __shared__ float sW[CO * 32 * KS * KS];
  __shared__ float sX[32 * KS * TW];
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

void launch_campp_conv2d(const CamppConv2d& a, int ks, hipStream_t st) {
  ZASR_REQUIRE(a.ci <= 32 && (ks == 1 || ks == 3), "campp conv2d: Ci <= 32, kernel 1 or 3");
  dim3 grid(cdiv(a.T, 64), a.fo, a.n);
  if (ks == 3) hipLaunchKernelGGL(campp_conv2d_kernel<3>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(campp_conv2d_kernel<1>, grid, dim3(256), 0, st, a);
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
  hipLaunchKernelGGL(campp_bnrelu_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st, x, ldx,
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
  hipLaunchKernelGGL(campp_im2col1d_kernel, dim3((unsigned)cdivl(n, 256)), dim3(256), 0, st, x,
                     ldx, N, Tin, Tout, C, K, stride, dil, pad, out);
}

// CAM context mask (CAMLayer.forward: context = mean_t(x) + seg_pooling(x); m = sigmoid(
// linear2(relu(linear1(context))))), block per (sequence n, segment g): 128 input channels
// (one per thread), the per-segment mask expanded to every frame of the segment:
// mexp[n * T + t][o] for t in segment g.  avg_pool1d(ceil_mode) divides a clipped last
// segment by its true length.
__global__ __launch_bounds__(128) void campp_cam_mask_kernel(CamppCamMask a) {
  __shared__ float sCtx[128];
  __shared__ float sZ[64];
  __shared__ float sM[32];
  const int tid = threadIdx.x, n = blockIdx.y, g = blockIdx.x;
  const int T = a.T, L = a.seg_len;
  const int s0 = g * L, s1 = min(T, s0 + L);
  const float* x = a.h + (long)n * T * 128 + tid;
  double tot = 0.0, seg = 0.0;
  for (int t = 0; t < T; ++t) {
    const float v = x[(long)t * 128];
    tot += v;
    if (t >= s0 && t < s1) seg += v;
  }
  sCtx[tid] = (float)(tot / T) + (float)(seg / (s1 - s0));
  __syncthreads();
  if (tid < 64) {
    float z = a.b1[tid];
    for (int c = 0; c < 128; ++c) z = fmaf(a.w1[tid * 128 + c], sCtx[c], z);
    sZ[tid] = fmaxf(z, 0.f);
  }
  __syncthreads();
  if (tid < 32) {
    float m = a.b2[tid];
    for (int c = 0; c < 64; ++c) m = fmaf(a.w2[tid * 64 + c], sZ[c], m);
    sM[tid] = 1.f / (1.f + expf(-m));
  }
  __syncthreads();
  for (int i = tid; i < (s1 - s0) * 32; i += 128) {
    const int t = s0 + i / 32, o = i % 32;
    a.mexp[((long)n * T + t) * 32 + o] = sM[o];
  }
}

void launch_campp_cam_mask(const CamppCamMask& a, hipStream_t st) {
  const int nseg = cdiv(a.T, a.seg_len);
  hipLaunchKernelGGL(campp_cam_mask_kernel, dim3(nseg, a.n), dim3(128), 0, st, a);
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
  hipLaunchKernelGGL(campp_stats_kernel, dim3(cdiv(N * C, 128)), dim3(128), 0, st, x, N, T, C, s,
                     b, out);
}

// per-utterance CMVN of fbank features: x[f][m] -= mean_f x[f][m] (one block per sequence,
// one thread per mel bin)
__global__ void campp_cmvn_kernel(float* __restrict__ x, const int* __restrict__ fr_off) {
  const int s = blockIdx.x, m = threadIdx.x;
  const int a = fr_off[s], e = fr_off[s + 1];
  if (m >= 80 || e <= a) return;
  double sum = 0.0;
  for (int f = a; f < e; ++f) sum += x[(long)f * 80 + m];
  const float mean = (float)(sum / (e - a));
  for (int f = a; f < e; ++f) x[(long)f * 80 + m] -= mean;
}

void launch_campp_cmvn(float* x, const int* fr_off, int nseq, hipStream_t st) {
  if (nseq <= 0) return;
  hipLaunchKernelGGL(campp_cmvn_kernel, dim3(nseq), dim3(128), 0, st, x, fr_off);
}

}  // namespace zasr
