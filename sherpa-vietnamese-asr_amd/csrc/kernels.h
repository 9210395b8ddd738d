// Launch wrappers for the non-GEMM kernels of the offline-ASR hot path.
//
// Ragged batches: every per-sequence tensor is stored packed, sequence after sequence,
// with a device offsets array `off[b]` (size B+1) per time resolution.  Kernels that
// need a row's sequence find it with a binary search over `off`.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace zasr {

// ---- fbank (core/asr_engine.py:698-721, kaldi semantics: SURVEY Appendix A) ----
struct FbankTables {
  const double* twiddle;    // [256][2]  exp(-2 pi i j / 512)
  const float* window;      // [400]     povey
  const int* mel_start;     // [80]
  const int* mel_len;       // [80]
  const int* mel_woff;      // [80] offset into mel_w
  const float* mel_w;       // packed triangle weights
};
// campp: the CAM++ front end (x 32768, snip_edges, signal-context pre-emphasis, floor 1.0;
// tables with the 20 Hz .. Nyquist mel bank) -- frames per sequence 1 + (n - 400) / 160
void launch_fbank(const float* wav, const long* wav_off, const int* nsamp, const int* fr_off,
                  int nseq, int total_frames, const FbankTables& tabs, float* out,
                  hipStream_t st, bool campp = false);

// the planner's silence detector (core/asr_engine.py:521-554): flags[f] = RMS of samples
// [f * frame_len, (f + 1) * frame_len) < threshold in numpy's float32 arithmetic, bit for bit;
// n / frame_len frames
void launch_silence_flags(const float* wav, long n, int frame_len, float threshold,
                          unsigned char* flags, hipStream_t st);

// a no-op kernel of block_threads threads through ZASR_LAUNCH, synchronised (zasr_selftest_launch)
void launch_selftest_noop(int block_threads);
// kernel self-tests on host operands (selftest.cpp; zasr_selftest_gemm_h3r / _ffn_h3 / _ffn_bf16)
void selftest_gemm_h3r(int M, int K, int N, int epi, const float* A, const float* W,
                       const float* bias, float* C);
void selftest_ffn_h3(int R, int D, int F, const float* Y, const float* W1, const float* b1,
                     const float* W2, const float* b2, const float* byp_orig,
                     const float* byp_scale, float* X);
void selftest_ffn_bf16(int R, int D, int F, const float* W1, const float* b1, const float* W2,
                       const float* b2, const float* byp_orig, const float* byp_scale, float* X,
                       int form);

// ---- CAM++ speaker embedding (campp_kernels.hip) ----
struct CamppConv2d {
  const float* x;      // [n][ci][fi][T]
  const float* w;      // [32][ci][ks][ks]
  const float* scale;  // [32] folded BN scale
  const float* shift;  // [32] folded BN shift
  const float* res;    // nullable residual [n][32][fo][T]
  float* y;            // [n][32][fo][T], or [n][T][32 * fo] (tdnn_out)
  int n, ci, fi, fo, T, sf;
  int relu, tdnn_out;
  int in_tf;           // x is the [n][T][fi] feature batch (ci = 1)
  const float* wk = nullptr;  // ci = 32: weights permuted by campp_conv2d_permute_weights
};
void campp_conv2d_permute_weights(const float* w, int ks, float* out);
void launch_campp_conv2d(const CamppConv2d& a, int ks, hipStream_t st);
void launch_campp_bnrelu(const float* x, int ldx, long R, int C, const float* s, const float* b,
                         float* y, hipStream_t st);
void launch_campp_im2col1d(const float* x, int ldx, int N, int Tin, int Tout, int C, int K,
                           int stride, int dil, int pad, float* out, hipStream_t st);
struct CamppCamMask {
  const float* h;      // [n * T][128] CAM input (nonlinear2 output)
  const float* w1;     // [64][128] linear1
  const float* b1;     // [64]
  const float* w2;     // [32][64] linear2
  const float* b2;     // [32]
  float* mexp;         // [n * T][32] mask per frame
  int n, T, seg_len;
};
void launch_campp_cam_mask(const CamppCamMask& a, hipStream_t st);
void launch_campp_stats(const float* x, int N, int T, int C, const float* s, const float* b,
                        float* out, hipStream_t st);
void launch_campp_cmvn(float* x, const int* fr_off, int nseq, hipStream_t st);
// window w = rows [win_row[w], + win_n[w]) of the packed fbank rows, zero-padded to wf frames
void launch_campp_gather(const float* rows, const int* win_row, const int* win_n, int nwin,
                         int wf, float* out, hipStream_t st);

// ---- ViBERT-capu encoder pieces (vibert_kernels.hip) ----
struct VibertEmbedArgs {
  const long* ids;    // [B * L]
  const long* tt;     // [B * L] token types
  const float* word;  // [V][H]
  const float* pos;   // [max_pos][H]
  const float* type;  // [types][H]
  const float* ln_g;
  const float* ln_b;
  float* x;           // [B * L][H]
  int L, H;
  float eps;
};
void launch_vibert_embed(const VibertEmbedArgs& a, long rows, hipStream_t st);
void launch_vibert_layernorm(float* x, long rows, int H, const float* g, const float* b, float eps,
                             hipStream_t st);
struct VibertAttnArgs {
  const float* qkv;   // [B * L][3 H]
  const long* mask;   // [B * L] attention_mask (0 = padding)
  float* ctx;         // [B * L][H]
  int L, H;
  float scale;        // 1 / sqrt(head dim)
};
void launch_vibert_attention(const VibertAttnArgs& a, int B, int heads, hipStream_t st);
void launch_vibert_gather(const float* x, const long* offsets, int B, int L, int W, int H, float* g,
                          hipStream_t st);

// ---- Silero VAD pieces (vad_kernels.hip) ----
struct VadFramesArgs {
  const float* audio;      // file mode: concatenated audio
  const long* off;         // [files] first sample of each file
  const long* win_start;   // [files] first window of each file in the job
  const unsigned* maxabs;  // [files] max |x| bits (auto boost) or nullptr
  const float* rows576;    // row mode: [windows][576] explicit inputs (else nullptr)
  float* frames;           // [windows * 4][256]
  int n_files;
};
void launch_vad_maxabs(const float* audio, const long* off, const long* len, int n_files,
                       unsigned* mx, hipStream_t st);
void launch_vad_frames(const VadFramesArgs& a, long n_windows, hipStream_t st);
void launch_vad_mag_im2col(const float* S, int ldS, int bins, int Kp, long n_windows, float* A,
                           hipStream_t st);
void launch_vad_im2col(const float* Y, long N, int T, int C, int stride, int Tout, float* A,
                       hipStream_t st);
struct VadLstmArgs {
  const float* gx;         // [windows][512] x W_ih^T + b_ih
  const float* whh;        // [512][128]
  const float* bhh;        // [512]
  const float* wd;         // [128] decoder conv weight
  float bd;
  const long* seg_start;   // [segments] first window whose probability the segment writes
  const int* seg_count;    // [segments] windows written
  const int* seg_warm;     // [segments] warm-up windows before seg_start, or nullptr
  const float* init;       // [segments][2][128] (h, c) at the first (warm-up) window, or nullptr
  float* s_out;            // [segments][2][128] state reached at seg_start, or nullptr
  float* e_out;            // [segments][2][128] final state, or nullptr
  float* probs;            // [windows]
};
void launch_vad_lstm(const VadLstmArgs& a, int n_segments, hipStream_t st);

// ---- Conv2dSubsampling pieces (icefall subsampling.py, 3P) ----
// conv.0 (1->8, 3x3, pad (0,1)) + SwooshR: fbank rows [T][80] -> [T-2][80][8]
// (out_bf16: bf16 output, native-exp/log SwooshR -- the bf16 mode; fast: f32 output with the
// native-exp/log SwooshR -- the f16x3 mode, whose GEMM epilogues use the same form)
void launch_conv1(const float* fb, const int* fb_off, const int* c1_off, const int* c1_map,
                  int total_rows, const float* w /*[8][9]*/, const float* b, void* out,
                  bool out_bf16, hipStream_t st, bool fast = false);
// ConvNeXt depthwise 7x7, zero padding per sequence: [L][19][128] -> [L][19][128]
// bf16 mode: out = x + pw2(SwooshL(pw1(dwconv7x7(x)))) (convnext_kernels.hip), x / out /
// ytmp (the depthwise output) bf16 [rows][19][128]; w1 / w2 the bf16 pw weights
void pack_frag32_host(const __bf16* w, int rows, int cols, __bf16* out);
// w1 / w2: pw1 [384][128] and pw2 [128][384] packed by pack_frag32_host
void launch_convnext_bf16(const void* x, const int* L_off, const int* L_map, int total_rows,
                          const float* dw_w, const float* dw_b, const void* w1, const float* b1,
                          const void* w2, const float* b2, void* ytmp, void* out,
                          hipStream_t st);
// f16x3: out = x + pw2(SwooshL(pw1(y) + b1)) + b2 in f32 over npos positions ([npos][128]
// each), the hidden layer on chip; w1p / w2p: the two fp16 pieces (hi, (w - hi) * 2^11) of
// pw1 / pw2, each packed by pack_frag32_host, piece t at offset t * 384 * 128 elements
void launch_convnext_mlp_h3(const float* y, const float* x, long npos, const void* w1p,
                            const float* b1, const void* w2p, const float* b2, float* out,
                            hipStream_t st);
// the same depthwise 7x7 (f32) on the tiled ConvNeXt kernel (convnext_kernels.hip, 32
// channels per block, staged values reused by up to 7 output frames); same FMA order per output
void launch_dwconv2d_tiled(const float* x, const int* L_off, const int* L_map, int total_rows,
                           const float* w, const float* b, float* out, hipStream_t st);

// ---- Zipformer2 encoder elementwise / per-sequence kernels ----
// y = x * exp(log_scale) * rsqrt(mean((x - bias)^2));  optionally y = orig + (y - orig) * s
// copy_out (nullable): the result also written there (the next layer's bypass input; may
// alias orig)
void launch_bias_norm(float* x, int rows, int d, const float* bias, float log_scale,
                      const float* orig, const float* bypass_scale, hipStream_t st,
                      float* copy_out = nullptr);
// x = orig + (x - orig) * s[c]
void launch_bypass(float* x, const float* orig, const float* s, long rows, int d, hipStream_t st);
// g[r][c] = x2[r][c] * sigmoid(x2[r][d + c])
void launch_glu(const float* x2, float* g, long rows, int d, hipStream_t st);
// g = x2[:, :d] * sigmoid(x2[:, d:]);  out[t][c] = SwooshR(b[c] + sum_k w[c][k] g[t+k-K/2][c]),
// zero padding per sequence
// the same depthwise conv + bias + SwooshR on an input that is already the GLU output
// ([rows][d], split modes: EPI_GLU in the in_proj GEMM)
void launch_dwconv1d_post_glu(const float* g, const int* off, const int* map, int total_rows,
                              int d, int K, const float* w, const float* b, float* out,
                              hipStream_t st);
void launch_dwconv1d_post_glu_bf16(const void* g, const int* off, const int* map,
                                   int total_rows, int d, int K, const float* w, const float* b,
                                   void* out, hipStream_t st);
void launch_glu_dwconv1d(const float* x2, const int* off, const int* map, int total_rows, int d,
                         int K, const float* w, const float* b, float* out, hipStream_t st);
// bf16 in (the conv in_proj output) / bf16 out (the conv out_proj input), bf16 mode
void launch_glu_dwconv1d_bf16(const void* x2, const int* off, const int* map, int total_rows,
                              int d, int K, const float* w, const float* b, void* out,
                              hipStream_t st);
// t1[r][c] = tanh(h3[r][c]) * h3[r][hid + c]
void launch_nonlin_prep(const float* h3, float* t1, long rows, int hid, hipStream_t st);
// SimpleDownsample: out[t'] = sum_u w[u] x[min(ds t' + u, L - 1)]
void launch_downsample(const float* x, const int* off_in, const int* off_out, const int* map_out,
                       int total_out, int d, int ds, const float* w_host8, float* out,
                       hipStream_t st);
// SimpleUpsample + out_combiner bypass: y[t] = orig[t] + (xd[t / ds] - orig[t]) * s
void launch_upsample_combine(const float* xd, const float* orig, const int* off_in,
                             const int* off_ds, const int* map_in, int total_rows, int d, int ds,
                             const float* s, float* y, hipStream_t st);
// seam between stacks: y = orig + (xd[t / ds] - orig) * s (ds == 1: y = orig) written as the
// next stack's input of width dn (truncated / zero-padded; null: none) and into columns
// [c0, d) of the full-dim output (null or c0 >= d: none); xd / off_ds unused when ds == 1
void launch_stack_glue(const float* xd, const float* orig, const int* off_in, const int* off_ds,
                       const int* map_in, int rows, int d, int ds, const float* s, float* next,
                       int dn, float* full, int ldf, int c0, hipStream_t st);
// row -> sequence index map for one resolution (off: [nseq + 1])
void launch_row2seq(const int* off, int nseq, int total, int* map, hipStream_t st);
// dst[r][0:dd] = src[r][0:min(ds, dd)], zero-padded  (convert_num_channels)
void launch_copy_cols(const float* src, int lds, int c0, float* dst, int ldd, int d0, int ncols,
                      long rows, bool zero_rest, int dst_width, hipStream_t st);

// ---- RelPositionMultiheadAttentionWeights: scores + softmax -> attention weights ----
struct AttnArgs {
  const float* qkp;        // [R][ (2*32+4) * H ]
  int H;                   // heads
  const float* pos_tab;    // [(2*Pmax - 1)][4*H]  linear_pos(pe(x)), row x + Pmax - 1
  int pmax;
  const int* row_off;      // [B+1] packed rows at this resolution
  const long* a_off;       // [B]   offset of sequence b's [H][L][ldA] block
  int nseq;
  int max_len;
  float* attn;             // normalised weights of heads < write_heads, [h][L][L4] per seq
  float* stats;            // [R][H][2]: row max, 1 / row sum
  int write_heads;
};
void launch_attn_softmax(const AttnArgs& a, hipStream_t st);
// bf16 mode, flash-style attention (attn_kernels.hip): qkp / v / out in bf16; the query
// and positional-query columns of qkp carry a log2(e) factor (folded into attn_in's bf16
// weights and bias at load).
//   mode 0: head-0 normalised weights in bf16, [L][L8] per sequence at a_off[b] (columns
//           [L, L8) zero; L8 = L rounded up to 8), the NonlinAttention GEMM operand
//   mode 1: self-attention with running statistics; writes out and stats_out
//   mode 2: self-attention with the statistics of mode 1 (stats_in)
//   mode 3: NonlinAttention fused, one online pass over head 0: running max / sum, the
//           unnormalised weights multiplied into t1 as they are computed (value accumulators
//           rescaled when the max moves), 1 / sum and * y in the epilogue; bf16 or f16x3
//           (pieces == kPiecesF16: fp16 pieces of the weights and of t1, one-accumulator
//           products, f32 y / z)
// stats: [R][H] c = row max + log2(row sum), log2 domain
struct AttnFlashArgs {
  const void* qkp;         // [R][68 H]: bf16 (pieces == 1) or f32
  int H;
  const float* pos_tab;    // [(2 pmax - 1)][4 H]
  int pmax;
  const int* row_off;      // [B+1]
  const long* a_off;       // [B] (mode 0)
  int nseq;
  int max_len;
  void* attn;              // mode 0: head 0's weights [L][L8] per sequence, bf16 / f32
  const void* v;           // [R][12 H], bf16 / f32
  void* out;               // [R][12 H], bf16 / f32
  const float* stats_in;   // mode 2
  float* stats_out;        // mode 1
  // 1: bf16 q / k / v / out / weights, log2(e) folded into q and p (the bf16 mode);
  // 2 / 3: f32 storage, every MFMA product split into 2 / 3 bf16 pieces per operand (the
  // bf16x3 / bf16x6 modes; q and p unscaled)
  int pieces = 1;
  // mode 3: NonlinAttention fused -- z = (A0 @ t1) * y with head 0's weights A0 consumed
  // where they are computed (never written): t1 as launch_nonlin_prep_t's transposed image
  // t1t[c][o8_b + j] (row stride ldt, zero-padded to L32; pieces == kPiecesF16: the fp16 hi
  // image, then the lo image at + hid * ldt), y [R][ldy] and z [R][hid]: bf16 in the bf16
  // mode (pieces == 1), f32 in the f16x3 mode
  const void* t1t = nullptr;
  const int* o8 = nullptr;
  int ldt = 0;
  int hid = 0;
  const void* y = nullptr;
  int ldy = 0;
  void* z = nullptr;
};
void launch_attn_flash(const AttnFlashArgs& a, int mode, hipStream_t st);
// t1t[c][o8_b + j] = bf16(tanh(h3[r][c]) * h3[r][hid + c]) for packed row r = off_b + j;
// columns [o8_b + L_b, o8_b + L8_b) zero; t1t row stride R8 = sum_b L8_b
// pieces > 1 (an f32 h3, the split modes): piece t of every value at t1t + t * hid * R8
void launch_nonlin_prep_t(const void* h3, bool h3_bf16, const int* off, const int* o8,
                          const int* map, int R, int hid, int R8, void* t1t, hipStream_t st,
                          int pieces = 1);
// fused self-attention consumer: out[:, 12h:12h+12] = softmax(S_h) V_h, recomputing S
struct AttnSAArgs {
  const float* qkp;
  int H;
  const float* pos_tab;
  int pmax;
  const int* row_off;
  int nseq;
  int max_len;
  const float* stats;      // [R][H][2] row max, 1 / row sum (read unless online)
  const float* v;          // [R][12H]
  float* out;              // [R][12H]
  float* stats_out;        // online: the statistics computed here, same layout
};
// online = running softmax statistics (first self-attention of a layer, writes stats_out);
// bf16 = QK^T / PV on bf16 MFMA (the bf16 precision mode)
void launch_attn_sa(const AttnSAArgs& a, bool online, bool bf16, hipStream_t st);

// ---- fused FeedforwardModule, bf16 mode (ffn_kernels.hip) ----
// X[R][D] += W2 SwooshL(W1 X + b1) + b2; W1 [F][D], W2 [D][F] bf16; D in {64, 96, 128, 192, 256}
bool ffn_fused_supported(int D);
void ffn_pack_host(const __bf16* w, int rows, int cols, __bf16* out);
void launch_ffn_fused(float* X, int R, int D, int F, const void* W1, const float* b1,
                      const void* W2, const float* b2, hipStream_t st,
                      const float* byp_orig = nullptr, const float* byp_scale = nullptr);
// f16x3 mode (f32-quality products, the hidden layer on chip as fp16 pieces): W1 / W2 as
// ffn_pack_h3_host images; D in {128, 256, 384, 512} with F % 32 == 0 or D = 192 with
// F % 64 == 0; every |w| < 31
// (ffn_h3_weights_ok: the kernel scales the weights' fp16 hi piece by 2^11)
bool ffn_h3_supported(int D, int F);
// development A/B switch of the f16x3 FFN's split barriers (default 1; 0: block barriers)
void ffn_h3_set_split(int on);
// the d = 384 bf16 FFN over per-CU row shares (ffn_rows_kernel): off unless ZASR_FFN_ROWS=1
void ffn_set_rows(int on);
int ffn_rows_on();
bool ffn_h3_weights_ok(const float* w, long n);
void ffn_pack_h3_host(const float* w, int rows, int cols, __bf16* out);
// Y (nullable): the rows the FFN reads when they are not X's own -- X += FFN(Y) (the ConvNeXt
// block's pointwise MLP on the depthwise conv's output, D = 128)
void launch_ffn_fused_h3(float* X, int R, int D, int F, const void* W1, const float* b1,
                         const void* W2, const float* b2, hipStream_t st,
                         const float* byp_orig = nullptr, const float* byp_scale = nullptr,
                         const float* Y = nullptr);

// ---- transducer search (core/asr_engine.py:1023-1153) ----
struct SearchState {
  // hypothesis slots, [S * Hmax]
  double* lp;
  int* lpf;           // 1: lp came from a non-cutoff log-add (np.float64 in the reference),
                      //    so the next frame adds it in f64; 0: a Python float, added in f32
  unsigned long long* hash;
  int* len;
  int* y1;            // newest context token (ys[-1], clamped >= 0)
  int* y2;            // older context token (ys[-2], clamped >= 0)
  int* hw;            // hotword automaton state
  int* node;          // last emission node (-1: none)
  int* nh;            // [S] live hypotheses
  // emission node pool, [S * node_cap]
  int* node_tok;
  int* node_frame;
  int* node_parent;
  double* node_lp;
  float4* node_stats;   // (entropy, sum p^(1/3), top1, top2) of the emitting joiner row
  int* node_count;      // [S]
  int node_cap;
};
struct HotwordTables {
  int num_states;       // 0 => no hotwords
  int num_cls;
  const int* tok2cls;   // [V] token -> column, -1 if the token is not in the trie
  const int* next;      // [states][cls]
  const double* delta;  // [states][cls]
  const double* node_score;  // [states]
};
struct DecoderW {
  const float* tap0;  // [V][D] grouped-conv tap 0 applied to each embedding row
  const float* tap1;  // [V][D] tap 1
  const float* bp;    // decoder_proj bias [D]
  int D;
};
struct DecJoinArgs {
  DecoderW dw;
  const float* wp;       // decoder_proj weight [D][D] (K contiguous)
  const int* y1;         // [S*H] slot contexts
  const int* y2;
  const float* enc;      // [sum T'][D]
  const int* enc_off;    // [S]
  void* J;               // [M][D] = tanh(enc[s, t] + dec[slot]), f32 or bf16 (j_bf16)
  int M, H, t;
  int j_bf16;
};
// live_t / live_len / live_f (optional): rows are (stream, window frame) = (r / live_f,
// r % live_f); a 32-row tile whose streams are all finished (live_t >= live_len) is skipped
struct JoinerArgs {
  const float* J;        // [M][D]
  const float* W;        // [V][D]
  const float* bias;     // [V]
  float* out;            // [M][V]
  int M, V, D;
  const int* live_t = nullptr;
  const int* live_len = nullptr;
  int live_f = 0;
  // split-bf16 modes: W_out as `pieces` bf16 pieces (piece t at Wx + t V D); J stays f32
  const __bf16* Wx = nullptr;
  int pieces = 0;
};
struct JoinerBf16Args {
  const __bf16* J;       // [M][D]
  const __bf16* W;       // [V][D]
  const float* bias;     // [V]
  float* out;            // [M][V]
  int M, V, D;
  const int* live_t = nullptr;
  const int* live_len = nullptr;
  int live_f = 0;
};
// Decoder-context table: the stateless decoder is a pure function of the two-token context
// (y_-2, y_-1) (core/asr_engine.py:1051-1056, 1072-1088 cache it per context), so the engine
// evaluates it once for all V^2 contexts at model load (8.2 GB f32 at V = 2000, D = 512 --
// small against 288 GB of HBM) and the search step turns a new hypothesis into the next
// frame's joiner input with one row gather:  J[slot] = tanh(enc[s, t + 1] + table[y2 V + y1]).
struct DecTable {
  const float* table;       // [V * V][D]
  int V;
  const float* enc;         // [sum T'][D]
  const int* enc_off;       // [S]
  const int* enc_len;       // [S]
  void* J;                  // [S*H][D] joiner input of the next frame (bf16 if j_bf16)
  int D;
  int j_bf16;
  int j_packed = 0;         // bf16 J in MFMA-fragment order (the packed joiner's A operand)
  // split-bf16 modes with j_packed: J = tanh() in f32 written as j_pieces bf16 pieces
  // (p0 = bf16(x), p1 = bf16(x - p0), ...), piece t at element offset t * j_plane
  int j_pieces = 0;
  long j_plane = 0;
};
// Speculative-greedy joiner on fragment-packed operands: J packed by the greedy search
// kernels ([row/32][D/16][64 lanes][8] bf16, rows padded to a multiple of 64), W packed once
// at load by gemm_rp_pack_weights ([col/32][D/16][64][8], zero beyond V).  One block per
// 64 x 64 output tile: both 64 KB operand tiles cross into LDS once with coalesced 16-byte
// loads (every load of the block in flight together), 4 waves x one 32 x 32 tile over all of D.
struct JoinerPackedArgs {
  const void* Jp;
  const void* Wp;
  const float* bias;   // [V]
  float* out;          // [M][V]
  int M, V, D;
  const int* live_t = nullptr;
  const int* live_len = nullptr;
  int live_f = 0;
  // split-bf16 modes: J and W as `pieces` packed images each (piece t of J at Jp + t j_plane,
  // of W at Wp + t w_plane, in bf16 elements); the logits are the f32 sum of the piece
  // products with u + v < pieces (joiner_split_packed_kernel)
  int pieces = 0;
  long j_plane = 0, w_plane = 0;
};
void launch_joiner_packed(const JoinerPackedArgs& j, hipStream_t st);
// *flag (device int) = 1 if any of the n floats of x is not finite, else 0
void launch_nonfinite_check(const float* x, long n, int* flag, hipStream_t st);
// rows the packed J buffer must hold for M joiner rows
inline long joiner_packed_rows(long M) { return (M + 63) / 64 * 64; }
void launch_search_init(const SearchState& s, int S, int Hmax, hipStream_t st);
void launch_decjoin(const DecJoinArgs& a, hipStream_t st);
void launch_joiner(const JoinerArgs& j, hipStream_t st);
void launch_joiner_bf16(const JoinerBf16Args& j, hipStream_t st);
// table[(y2 V + y1) D + n] = decoder_proj(relu(conv(E[y2], E[y1])))[n], all V^2 contexts
void launch_dec_table(const DecoderW& dw, const float* wp, int V, float* table, hipStream_t st);
// J of frame 0 for slot 0 of every stream (context (0, 0))
void launch_table_init(const DecTable& dt, int S, int Hmax, hipStream_t st);
// dt == nullptr: the next frame's J comes from launch_decjoin
void launch_search_step(const SearchState& s, const float* logits, int V, int S, int Hmax,
                        int beam, int t, const int* enc_len, const HotwordTables& hw,
                        const DecTable* dt, hipStream_t st);
// ---- speculative greedy search (beam 1 with the decoder-context table) ----
// Greedy keeps the decoder context across blank frames, so the joiner rows of the next F
// frames of a stream are all known until the first emission.  One super-step = the joiner
// over [S][F] rows (J rows written by the previous super-step) + greedy_spec: per stream,
// the exact per-frame top-1 of the frame-by-frame step (same f32 score arithmetic, same
// smaller-index tie break) for every frame of the window under the all-blank-so-far
// hypothesis, then the first non-blank frame (if any) is the emission; t_cur advances past
// it (or by the window).  Streams still running after the step add 1 to active[parity].
// J layout: [S][F][D] (row s * F + f = frame t_cur[s] + f).
void launch_greedy_spec_init(const DecTable& dt, int S, int F, int* t_cur, int* active,
                             hipStream_t st);
void launch_greedy_spec(const SearchState& s, const float* logits, int V, int S, int F,
                        int* t_cur, const int* enc_len, const HotwordTables& hw,
                        const DecTable& dt, int* active, int parity, hipStream_t st);
// One launch per super-step (joiner_greedy_kernel): the packed joiner over row tiles of 8
// streams x 4 frames, and in each row tile's last-arriving block (an agent-scope arrival
// counter; logits handed over by write-through stores and loads) that tile's greedy step,
// one wave per stream -- the same logits bit for bit (same MFMA sequence per 32 x 32 tile)
// and the same per-frame arithmetic as joiner + greedy_spec, without the second launch and
// its boundary.  F = 4.  `out` rows have stride ldo (>= V, a multiple of 32); cnt: one int
// per row tile, zero before the first launch (each tile's last block re-zeroes it).
struct GreedyFusedArgs {
  JoinerPackedArgs j;  // j.out = logits [S * 4][ldo], j.M = S * 4
  int ldo;
  SearchState st;
  int* t_cur;
  const int* enc_len;
  HotwordTables hw;
  DecTable dt;
  int* active;
  int parity;
  int* cnt;
  int S;
};
void launch_joiner_greedy(const GreedyFusedArgs& a, hipStream_t st);
inline int joiner_greedy_ldo(int V) { return (V + 31) / 32 * 32; }
void launch_search_final(const SearchState& s, int S, int Hmax, const HotwordTables& hw,
                         int out_cap, int* out_tok, int* out_frame, double* out_lp,
                         float4* out_stats, int* out_count, hipStream_t st);

}  // namespace zasr
