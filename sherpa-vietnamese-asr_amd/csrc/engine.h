// Host runtime of libzasr: device-resident model, per-batch workspace, and the encoder /
// search drivers that sequence the HIP kernels on one stream.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gemm.h"
#include "kernels.h"

namespace zasr {

struct ModelConfig {
  std::string name;
  std::vector<int> dims, layers, ff, heads, ds, kernels;
  int qd = 32, vd = 12, pd = 4, pos_dim = 48;
  int V = 0, dec_dim = 0, joiner_dim = 0, context = 2;
  int c1 = 8, c2 = 32, c3 = 128;
  int max_dim() const {
    int m = 0;
    for (int d : dims) m = d > m ? d : m;
    return m;
  }
};

struct DLin {
  float* w = nullptr;  // [N][K]
  float* b = nullptr;  // [N] or null
  int N = 0, K = 0;
  void* wh = nullptr;  // bf16 copy of w (precision mode bf16)
  float* bh = nullptr; // bias of the bf16 path when it differs from b (folded row scales)
  void* wp = nullptr;  // bf16 in MFMA-fragment order (ffn_pack_host), the wide fused FFN's operand
  void* wx = nullptr;  // split bf16 of w (precision mode bf16x3): hi [N][K], then lo [N][K]
  void* wr = nullptr;  // f16x3: the two fp16 pieces in MFMA-fragment order (gemm_h3r)
  // split modes, the conv modules' in_proj: rows (and bias) interleaved so output columns
  // 2c / 2c + 1 are the GLU halves of channel c -- the GEMM epilogue applies the GLU (EPI_GLU)
  bool glu = false;
};

struct DLayer {
  DLin attn_in, sa_in[2], sa_out[2], ff_in[3], ff_out[3], na_in, na_out, cv_in[2], cv_out[2];
  float* cv_dw_w[2] = {nullptr, nullptr};
  float* cv_dw_b[2] = {nullptr, nullptr};
  float* bypass = nullptr;
  float* bypass_mid = nullptr;
  float* norm_b = nullptr;
  float norm_ls = 0.f;
  std::vector<float> pos_w;  // linear_pos weight [4h][pos_dim] (host, to rebuild tables)
  float* pos_tab = nullptr;  // [(2*pmax-1)][4h]
};

struct DStack {
  int d = 0, F = 0, h = 0, ds = 1, K = 0;
  float ds_w[8] = {0};
  float* comb = nullptr;  // out_combiner bypass scale
  std::vector<DLayer> layers;
};

struct DModel {
  ModelConfig cfg;
  float *conv0_w = nullptr, *conv0_b = nullptr;
  DLin conv4, conv7, pw1, pw2, out, enc_proj, dec_proj, joiner;
  float *dw_w = nullptr, *dw_b = nullptr;
  float* out_norm_b = nullptr;
  float out_norm_ls = 0.f;
  std::vector<DStack> stacks;
  float out_ds_w[2] = {0, 0};
  float* dec_emb = nullptr;   // [V][D]
  float* dec_conv = nullptr;  // [D][4][2]
  void* joiner_packed = nullptr;  // bf16 joiner weights in MFMA-fragment order (bf16 mode),
                                  // or their split pieces (bf16x3 / bf16x6), one image each
  long joiner_plane = 0;          // bf16 elements per packed piece image
  float* dec_table = nullptr;  // [V*V][D] decoder output per context (null: too large)
  float* dec_tap0 = nullptr;  // [V][D] conv tap 0 of each embedding row
  float* dec_tap1 = nullptr;  // [V][D] conv tap 1
  int pmax = 0;
  std::vector<void*> allocations;
};

struct HotwordDFA {
  int num_states = 0, num_cls = 0;
  std::vector<int> tok2cls, next;
  std::vector<double> delta, node_score;
};
HotwordDFA build_hotword_dfa(const std::vector<std::vector<int>>& phrases,
                             const std::vector<float>& scores, int V);

struct TokenResult {
  std::vector<int> tok, frame;
  std::vector<double> lp;
  std::vector<float> stats;  // 4 per token
  int t_out = 0;
};

class Engine {
 public:
  // model_dir: config.json + model.safetensors or the reference's ONNX files (onnx_io.h);
  // hotwords: token-id phrases + scores, compiled into the device automaton once V is known
  Engine(const std::string& model_dir, int device, int beam, bool greedy,
         const std::vector<std::vector<int>>& hotwords, const std::vector<float>& hotword_scores,
         int precision);
  ~Engine();

  int vocab() const { return model_.cfg.V; }
  int joiner_dim() const { return model_.cfg.joiner_dim; }
  int default_beam() const { return beam_; }
  hipStream_t stream() const { return stream_; }

  // full path from device waveforms (packed); results in chunk order
  std::vector<TokenResult> decode_device(const float* d_wav, const std::vector<long>& wav_off,
                                         const std::vector<long>& n, int beam, hipStream_t st);
  // several batches back to back (results in chunk order, batch_sizes[i] chunks per batch):
  // batch k+1's fbank + encoder run on the call's stream while batch k's search runs on the
  // engine's high-priority search stream -- the search loop is latency-bound on few CUs, so
  // the encoder of the next batch fills the rest of the chip
  std::vector<TokenResult> decode_device_batches(const float* d_wav, const std::vector<long>& wav_off,
                                                 const std::vector<long>& n,
                                                 const std::vector<int>& batch_sizes, int beam,
                                                 hipStream_t st);
  // the same pipeline from HOST waveforms (h_wav: pinned memory for an asynchronous copy):
  // each batch's span of samples is copied into its encoder slot's device buffer on the
  // engine's copy stream and its fbank waits on that copy only, so batch k + 1's upload runs
  // under batch k's encoder / search (the reference's unit of work starts from host audio,
  // core/asr_engine.py:2068)
  std::vector<TokenResult> decode_host_batches(const float* h_wav, const std::vector<long>& wav_off,
                                               const std::vector<long>& n,
                                               const std::vector<int>& batch_sizes, int beam,
                                               hipStream_t st);
  std::vector<TokenResult> decode_features(const std::vector<const float*>& feats,
                                           const std::vector<long>& frames, int beam);
  void fbank_host(const float* wav, long n, float* out);
  void encode_host(const std::vector<const float*>& feats, const std::vector<long>& frames,
                   std::vector<float>& out, std::vector<int>& t_out);
  std::vector<TokenResult> search_host(const std::vector<const float*>& enc,
                                       const std::vector<long>& t_out, int beam);

  // profiling
  // mode 0: off, 1: kernel classes, 2: classes with the GEMMs split by shape
  void profile_enable(int mode) {
    prof_on_ = mode > 0;
    prof_shapes_ = mode == 2;
  }
  void profile_reset();
  std::string profile_report();

  // which kernel each part of the model was routed to at load (JSON; zasr_model_routes): in
  // f16x3 a layer whose weights reach 31 in magnitude keeps the two-accumulator GEMMs
  // (ffn_h3_weights_ok), and a vocabulary whose V^2 D decoder table exceeds the size limit runs
  // the per-frame decoder (decjoin_kernel)
  std::string routes_json() const;
  // replace the fbank's 80 triangular filters (row-major [80][n_bins] weights over the FFT's
  // power bins, n_bins 256 or 257 with bin 256 zero): the reference's browser fbank uses Hz
  // triangles (offline_pwa/static/js/pure-ort-asr-worker.js:369-397) where knf uses mel ones
  void set_mel_banks(const float* banks, int n_bins);

  std::mutex mu;

 private:
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
  };
  template <class T>
  T* ws(const std::string& name, size_t count);
  void upload(void* dst, const void* src, size_t bytes);

  // a batch whose encoder output is enqueued (enc_out slot `slot`), waiting for its search
  struct Pending {
    int B = 0;
    std::vector<int> valid, t_out;
    float* enc = nullptr;
    hipEvent_t ready = nullptr;
  };
  // out_slot: encoder output buffer, completion event and pinned arena (0..kMaxEnc);
  // ws_slot: encoder workspace set (0..kMaxEnc-1) -- several batches' encoders may run at
  // once on separate streams
  void encode_stage(const float* d_wav, const std::vector<long>& wav_off, const std::vector<long>& n,
                    int out_slot, int ws_slot, hipStream_t stream, Pending& p);
  std::vector<TokenResult> search_stage(Pending& p, int beam);
  // decode_device_batches for beam search: several batches' searches in flight
  std::vector<TokenResult> decode_batches_two_searches(const float* d_wav,
                                                       const std::vector<long>& wav_off,
                                                       const std::vector<long>& n,
                                                       const std::vector<int>& batch_sizes,
                                                       int beam, hipStream_t main_st);
  // pinned staging for host->device metadata uploads: one arena per encoder output slot
  // plus one for the search, so an upload never waits for the stream to drain
  struct PinArena {
    char* p = nullptr;
    size_t cap = 0, used = 0, want = 0;
  };
  static constexpr int kMaxEnc = 3;  // encoder streams of the batch pipeline
  // kMaxEnc + 1 output slots, then one per search job set (two beam searches in flight)
  static constexpr int kMaxJobs = 3;  // beam searches in flight
  PinArena pin_[kMaxEnc + 1 + kMaxJobs];
  std::string ws_tag_;  // workspace-name prefix of the encoder workspace set in use
  int pin_cur_ = 0;
  void pin_reset(int arena);

  // pipeline stages (all on st_)
  void run_fbank(const float* d_wav, const std::vector<long>& wav_off, const std::vector<long>& n,
                 float* d_feats, std::vector<int>& frames);
  void run_encoder(const float* d_feats, const std::vector<int>& T, float* d_enc,
                   std::vector<int>& t_out);
  std::vector<TokenResult> run_search(const float* d_enc, const std::vector<int>& t_out, int beam);
  // a search whose launches and result copies are enqueued; collect_search waits for it.
  // Job set `set` (0 .. kMaxJobs - 1) owns its search workspace, pinned arena, result buffers and
  // completion event, so two jobs can be in flight on the two search streams.
  struct SearchJob {
    int S_all = 0, S = 0, cap = 0, set = 0, Tmax = 0;
    std::vector<int> order, t_out;
    bool check_finite = false;  // f16x3: the encoder output's fp16-range guard
    hipStream_t stream = nullptr;
  };
  void launch_search(const float* d_enc, const std::vector<int>& t_out, int beam, int set,
                     hipStream_t stream, bool split_groups, SearchJob& job);
  std::vector<TokenResult> collect_search(SearchJob& job);
  struct ResPin {  // pinned host result buffers of one job set
    char* p = nullptr;
    size_t cap = 0;
  };
  ResPin res_pin_[kMaxJobs];
  void layer_forward(const DStack& stk, const DLayer& ly, float* X, int R, const int* d_off,
                     const int* d_map, const std::vector<int>& lens, const long* d_aoff,
                     const void* d_slices_nl, int maxL, const int* d_o8, int R8, bool orig_ready = false,
                     bool last_layer = true);
  // byp_orig / byp_scale (split modes, EPI_RESADD): bypass_mid in the epilogue
  void linear(const DLin& l, const float* A, int lda, int M, float* C, int ldc, int epi,
              const char* cls = "enc_gemm", const float* byp_orig = nullptr,
              const float* byp_scale = nullptr);
  // bf16 mode only: A and/or C in bf16 (GEMM -> GEMM intermediates; the GEMM rounds A to
  // bf16 on load anyway, so storing it rounded changes nothing numerically)
  void linear_h(const DLin& l, const void* A, bool a_bf16, int lda, int M, void* C, bool c_bf16,
                int ldc, int epi, const float* byp_orig = nullptr,
                const float* byp_scale = nullptr);
  void ensure_pos_tables(int max_len);

  // timing
  struct ProfEvent {
    std::string name;
    hipEvent_t a, b;
  };
  void prof_begin(const char* name);
  void prof_begin(const std::string& name);
  void prof_end();
  static std::string shape_key(const char* cls, int M, int K, int N, bool w16, bool a16,
                               bool c16, int epi);
  bool prof_on_ = false;
  bool prof_shapes_ = false;  // GEMM classes split by shape (profile mode 2)
  std::vector<ProfEvent> prof_pending_;
  std::map<std::string, std::pair<long, double>> prof_acc_;
  std::vector<hipEvent_t> event_pool_;
  hipEvent_t take_event();

  DModel model_;
  struct Routes {
    int ffn_fused_h3 = 0, ffn_gemm_pair = 0;  // f16x3 FFNs (d 128..512): fused / GEMM pair
    int gemm_h3r = 0, gemm_x3_range = 0;      // f16x3 layer projections the row-resident GEMM
                                              // shapes admit: taken / refused by the range check
    int cnx_ffn_h3 = -1;                      // f16x3 ConvNeXt MLP fused (1) or not (0); -1 n/a
  } routes_;
  int device_ = 0;
  int beam_ = 8;
  [[maybe_unused]] bool greedy_ = false;
  // make main_st wait for every encoder stream of a batch pipeline that is not main_st
  void order_after_encoders(const hipStream_t* enc_st, int E, hipStream_t main_st);
  int precision_ = 0;
  // bf16 pieces per operand of the split-bf16 modes (bf16x3: 2, bf16x6: 3), 0 otherwise
  // the `pieces` code of the split modes: 2 / 3 bf16 pieces (bf16x3 / bf16x6), kPiecesF16
  // for the two fp16 pieces of f16x3 (gemm.h); 0 otherwise
  int split_pieces() const {
    return precision_ == 3 ? 2 : precision_ == 4 ? 3 : precision_ == 5 ? kPiecesF16 : 0;
  }
  hipStream_t stream_ = nullptr;
  hipStream_t stream2_ = nullptr;  // searches (high priority: overlaps the next batch's encoder)
  hipStream_t stream3_ = nullptr;  // the second group of a beam search (high priority)
  hipStream_t stream4_ = nullptr;  // the third beam search in flight (high priority)
  int search_cus_ = 0;             // > 0: search / encoder streams on disjoint CU sets
  hipStream_t enc_extra_[kMaxEnc - 1] = {};  // encoder streams 1.. of the batch pipeline
  // [0, kMaxEnc]: encoder output slots; kMaxEnc + 1: search done; kMaxEnc + 2: start;
  // kMaxEnc + 3: beam groups; kMaxEnc + 4 + set: search job `set` complete
  hipEvent_t part_ev_[kMaxEnc + 4 + kMaxJobs] = {};
  hipStream_t st_ = nullptr;  // stream of the current call
  // decode_host_batches: the call's waveforms are host memory; encode_stage uploads each
  // batch's span on copy_st_ (upload_ev_[slot]: that slot's copy done)
  const float* host_wav_ = nullptr;
  hipStream_t copy_st_ = nullptr;
  hipEvent_t upload_ev_[kMaxEnc + 1] = {};
  std::map<std::string, Buf> ws_;
  // fbank tables
  double* d_twiddle_ = nullptr;
  float* d_window_ = nullptr;
  int* d_mel_meta_ = nullptr;  // start[80], len[80], woff[80]
  float* d_mel_w_ = nullptr;
  int* h_pinned_ = nullptr;  // pinned host word (live-stream count of the greedy search)
  // hotword tables
  HotwordDFA hw_host_;
  HotwordTables hw_{};
};

}  // namespace zasr
