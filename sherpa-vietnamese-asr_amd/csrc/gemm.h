// Dense projection GEMMs of the Zipformer transducer on CDNA4 MFMA.
//
//   C[m, n] = epi( alpha * sum_k A'[m, k] * B[k, n] + bias[n] )
//
// A' is produced by an A-loader (plain row-major activations, the joiner's
// tanh(enc + dec) prologue, or implicit im2col for the Conv2dSubsampling convs), B is a
// weight matrix [N][K] (K contiguous, the nn.Linear layout) or an activation matrix [K][N]
// (N contiguous: the attention values).  Batched launches carry one descriptor per
// z-slice (a sequence, or a (sequence, head) pair) so ragged sequences never pad.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace zasr {

enum GemmEpi : int {
  EPI_NONE = 0,     // C = v
  EPI_SWOOSHL = 1,  // C = SwooshL(v)
  EPI_SWOOSHR = 2,  // C = SwooshR(v)
  EPI_RESADD = 3,   // C += v          (residual: src = src + module(src))
  EPI_MULAUX = 4,   // C = v * aux[m, n]
  EPI_MULAUX16 = 5, // C = v * aux[m, n], aux bf16 (gemm_bf16 only)
  EPI_RELU = 6,     // C = max(v, 0)  (gemm_f32 only: CAM++ TDNN layers, BN folded in)
  EPI_GELU = 7,     // C = v * Phi(v) = 0.5 v (1 + erf(v / sqrt 2))  (gemm_f32 only: ViBERT FFN)
  EPI_GLU = 8,      // C[m, n / 2] = v[2c] * sigmoid(v[2c + 1]) (gemm_x3 only: the conv modules'
                    // in_proj with interleaved weight rows; N = 2 x the output width, ldc = N / 2)
};

enum GemmALoad : int {
  ALOAD_DENSE = 0,   // A[m * lda + k]
  ALOAD_JOINER = 1,  // retired (the joiner has its own split-K kernels)
  ALOAD_CONV2 = 2,   // im2col of conv1 output [T1][80][8]   -> conv.4 (3x3, stride 2)
  ALOAD_CONV3 = 3,   // im2col of conv2 output [L2][39][32]  -> conv.7 (3x3, stride (1,2))
  ALOAD_BNRELU = 4,  // max(A[m * lda + k] * a_scale[k] + a_shift[k], 0)  (gemm_f32 only)
  ALOAD_IM2COL1D = 5,  // 1-D conv im2col over sequences, see GemmIm2col1d  (gemm_f32 only)
};
// ALOAD_IM2COL1D: row m = n * Tout + t, column k = q * C + c reads
// A[(n * Tin + t * stride + q * dil - pad) * lda + c], 0 outside [0, Tin).  C % 4 == 0.
struct GemmIm2col1d {
  int Tin = 0, Tout = 0, C = 0, stride = 1, dil = 1, pad = 0;
};

// Per z-slice descriptor (device array).  Offsets are in elements.
struct GemmSlice {
  long a_off;
  long b_off;
  long c_off;
  long aux_off;
  int M;
  int K;
  int lda;
  int pad_;
};

struct JoinerALoad {
  const float* enc;      // [sum T', D]
  const float* dec;      // [S*H, D]
  const int* enc_off;    // [S] first encoder row of stream s
  const int* enc_len;    // [S] T'_s
  int H;                 // hyp slots per stream
  int t;                 // current frame
};

struct GemmParams {
  const float* A;
  int lda;
  const float* B;
  long sbk, sbn;         // B element (k, n) = B[k * sbk + n * sbn]
  float* C;
  int ldc;
  const float* bias;     // [N] or nullptr
  const float* aux;      // EPI_MULAUX operand
  int ldaux;
  int M, N, K;
  float alpha;
  const GemmSlice* slices;  // nullptr => single problem with the fields above
  int num_slices;
  int max_M;                // max M over slices (grid sizing)
  // EPI_RESADD in gemm_bf16 and gemm_x3 (nullable): after the residual add, the layer's mid bypass
  // C = orig + (C - orig) * scale[n] (orig row stride ldc)
  const float* byp_orig = nullptr;
  const float* byp_scale = nullptr;
  JoinerALoad joiner;
  const float* a_scale = nullptr;  // ALOAD_BNRELU
  const float* a_shift = nullptr;
  GemmIm2col1d i2c;                // ALOAD_IM2COL1D
};

// Launch; picks a tile shape from (max_M, N).  B_ncontig selects the [K][N] B layout.
void gemm_f32(const GemmParams& p, int epi, int aload, bool b_ncontig, hipStream_t stream);
// bf16-input variant: Bw = bf16 weights [N][K] (K contiguous, row stride p.sbn elements);
// A = f32 activations rounded to bf16 while staging (or bf16 when a_bf16: p.A then points
// at __bf16 data); f32 accumulate and epilogue; C written as f32 (or bf16 when c_bf16).
// Requires N, ldc (and ldaux for EPI_MULAUX) to be multiples of 4.

void gemm_bf16(const GemmParams& p, const void* Bw, int epi, int aload, hipStream_t stream,
               bool a_bf16 = false, bool c_bf16 = false);

// Row-panel GEMM (gemm_rp.hip) for K in {48, 64, 96, 128, 144, 192, 256, 288, 384, 512}:
// C = epi(A W^T + bias) with W pre-packed by gemm_rp_pack_weights (bf16 [N][K] ->
// MFMA-fragment order, gemm_rp_packed_elems(N, K) bf16 elements).  Combinations: A f32 -> C
// bf16 (EPI_NONE / EPI_SWOOSHL), A f32 -> C f32 (EPI_NONE), A bf16 -> C f32 (EPI_RESADD).
// Returns false (nothing launched) for any other combination or shape.
bool gemm_rp_supported_k(int K);
long gemm_rp_packed_elems(int N, int K);
void gemm_rp_pack_weights(const void* W_bf16, int N, int K, void* out, hipStream_t stream);
bool gemm_rp(const void* A, bool a_bf16, int lda, const void* Bp, const float* bias, void* C,
             bool c_bf16, int ldc, int M, int N, int K, int epi, hipStream_t stream);

// Split-bf16 variant (gemm_x3.hip; the "bf16x3" / "bf16x6" precision modes): A f32 (dense,
// or the implicit-im2col loaders ALOAD_CONV2 / ALOAD_CONV3) split into `pieces` bf16 pieces
// while staging; W pre-split by split_to_bf16, piece t at Bw + t * b_lo elements; C f32.
// pieces = 2: 3 MFMAs per product (~2^-16 relative); pieces = 3: 6 MFMAs (exact-f32
// quality); pieces = kPiecesF16: the f16x3 format, two fp16 pieces hi + lo * 2^-11 per
// operand and 3 fp16 MFMAs per product (~2^-22 relative, two accumulators; operands below
// 65504).  Epilogues NONE, SWOOSHL, SWOOSHR, RESADD, MULAUX (f32 aux).  N, ldc (and ldaux)
// multiples of 4; K a multiple of 8 for dense A.
// the `pieces` code of the f16x3 format (two fp16 pieces stored; see gemm_dev.h split_h8)
constexpr int kPiecesF16 = 4;
// pieces stored per operand for a `pieces` code
inline int stored_pieces(int pieces) { return pieces == kPiecesF16 ? 2 : pieces; }
void gemm_x3(const GemmParams& p, const void* Bw, long b_lo, int epi, int aload, hipStream_t stream,
             int pieces);
// f16x3 projection GEMM with the A row tile resident on chip (gemm_h3r.hip): A f32 [M][K]
// (lda = K), W as two fp16 pieces in MFMA-fragment order (ffn_pack_h3_host, every |w| < 31),
// C f32; epilogues NONE, RESADD, GLU (ldc = N / 2).  K in {96, 192, 256, 288, 384, 512},
// N >= 128, N % 16 == 0.
bool gemm_h3r_supported(int K, int N, int epi);
void gemm_h3r(const float* A, const void* Wp, const float* bias, float* C, int ldc, int M, int N,
              int K, int epi, hipStream_t stream);
// dst[t * n + i] = piece t of src[i]: bf16(src[i] - sum of the previous pieces), t < pieces
void split_to_bf16(const float* src, void* dst, long n, int pieces, hipStream_t stream);

// device f32 -> bf16 (round to nearest even) copy
void convert_to_bf16(const float* src, void* dst, long n, hipStream_t stream);
// dst[r][k] = bf16(src[r][k] * row_scale[r]) (one rounding), src / dst [N][K]
void convert_rows_to_bf16(const float* src, const float* row_scale, void* dst, long N, int K,
                          hipStream_t stream);

}  // namespace zasr
