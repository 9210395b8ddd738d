/*
 * zasr.h — C ABI of libzasr.so, the MI355X-native offline-ASR hot path
 * (kaldi fbank -> Zipformer2 transducer encoder -> stateless decoder + joiner ->
 *  greedy / modified-beam search with Aho-Corasick hotword biasing).
 *
 * Plain C types only: caller-owned input buffers are read during the call; results are
 * library-owned until zasr_result_free (mirrors SherpaOnnxDestroyOfflineStreamResultJson,
 * offline_pwa/static/vendor/sherpa-onnx-wasm/sherpa-onnx-asr.js:1872-1878).  Every entry
 * point returns 0 on success and a nonzero code on failure; zasr_last_error() gives the
 * message of the calling thread's last failure.  One handle may be used from several
 * host threads (calls on a handle are serialised internally), matching the reference's
 * two decode workers sharing one set of sessions (core/asr_engine.py:2291-2315).
 *
 * Reference interfaces each entry point replaces:
 *   zasr_create            core/asr_engine.py:903-1020 create_recognizer (ORT sessions,
 *                          tokens, hotword ContextGraph); sherpa-onnx
 *                          SherpaOnnxCreateOfflineRecognizer (sherpa-onnx-asr.js:1782)
 *   zasr_destroy           SherpaOnnxDestroyOfflineRecognizer; core/asr_engine.py:743-773
 *                          clear_model_cache
 *   zasr_fbank             core/asr_engine.py:698-721 compute_fbank_ort (kaldi-native-fbank)
 *   zasr_decode_batch      core/asr_engine.py:1209-1226 decode_chunk (fbank + search) over a
 *                          batch of chunks; SherpaOnnxAcceptWaveformOffline +
 *                          SherpaOnnxDecodeOfflineStream (sherpa-onnx-asr.js:1799-1830)
 *   zasr_decode_features   core/asr_engine.py:1224 _ort_beam_search with precomputed
 *                          features (ROVER shares one fbank, core/asr_engine.py:2346-2350)
 *   zasr_encode_features   the encoder session run, core/asr_engine.py:1045-1049
 *   zasr_silence_flags     core/asr_engine.py:521-554 find_silent_regions (the planner's
 *                          frame energies, numpy float32 bit for bit; regions on the host)
 *   zasr_search_encoder_out  the search loop alone, core/asr_engine.py:1051-1153
 *   zasr_result_*          the (token_ids, frames, ys_log_probs, T, emit_logits) tuple of
 *                          core/asr_engine.py:1153 (entropy statistics instead of raw
 *                          logits rows, reduced on device); SherpaOnnxGetOfflineStreamResult
 */
#ifndef ZASR_H_
#define ZASR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct zasr_recognizer zasr_recognizer;
typedef struct zasr_result zasr_result;

enum {
  ZASR_OK = 0,
  ZASR_ERR_INVALID = 1,   /* bad argument */
  ZASR_ERR_NOT_FOUND = 2, /* missing model file (reference raises FileNotFoundError) */
  ZASR_ERR_RUNTIME = 3,   /* HIP / internal failure */
};

/* FP32: exact-f32 MFMA everywhere (parity mode).  BF16: bf16 MFMA operands for the encoder
   projections / attention and the joiner, f32 accumulate, norms and search.  BF16_ENC: the
   BF16 encoder with the f32 joiner and search of FP32 (no bf16 rounding of the joiner input).
   BF16X3: f32 storage as FP32, every encoder projection product as three bf16 MFMAs over
   hi / lo operand halves (relative product error ~2^-16).  BF16X6: three bf16 pieces per
   operand, six MFMAs per product (dropped terms below 2^-24: exact-f32 quality at bf16 MFMA
   rates; token-exact against the fp32 oracle).  F16X3: two fp16 pieces
   per operand, hi = fp16(x) and lo = fp16((x - hi) * 2^11), three fp16 MFMAs per product
   (hi*hi + (hi*lo + lo*hi) * 2^-11, ~2^-22 relative: f32 quality at half the MFMAs of
   BF16X6); operands must stay below 65504 in magnitude (the 68M model's stay below 30). */
enum {
  ZASR_PRECISION_FP32 = 0,
  ZASR_PRECISION_BF16 = 1,
  ZASR_PRECISION_BF16_ENC = 2,
  ZASR_PRECISION_BF16X3 = 3,
  ZASR_PRECISION_BF16X6 = 4,
  ZASR_PRECISION_F16X3 = 5
};

typedef struct zasr_config {
  const char* model_dir;        /* config.json + model.safetensors, or the reference's
                                   encoder-/decoder-/joiner-*.onnx (+ tokens.txt for hosts) */
  const char* decoding_method;  /* "greedy_search" | "modified_beam_search" */
  int32_t max_active_paths;     /* beam for modified_beam_search, 1..16 (reference: 8) */
  float blank_penalty;          /* must be 0 (the reference applies none) */
  /* hotwords as token-id phrases (sentencepiece encoding stays on the host,
     core/hotword_context.py:234-248); may be NULL / 0 */
  const int32_t* hotword_tokens;  /* concatenated phrases */
  const int32_t* hotword_lens;    /* per-phrase token counts */
  const float* hotword_scores;    /* per-phrase score (reference default 1.5) */
  int32_t num_hotwords;
  int32_t device_id;            /* HIP device ordinal */
  int32_t precision;            /* ZASR_PRECISION_* */
} zasr_config;

int zasr_create(const zasr_config* cfg, zasr_recognizer** out);
void zasr_destroy(zasr_recognizer* h);

/* Host-only (no GPU): load a model directory the way zasr_create does -- config.json +
   model.safetensors, or the reference's encoder-/decoder-/joiner-*.onnx set chosen like
   create_recognizer (core/asr_engine.py:913-928: non-int8 preferred, int8 dequantized when it
   is the only file) with the architecture inferred from the initializer shapes -- and write
   out_dir/config.json + out_dir/model.safetensors (float32, the engine's tensor names).
   Replaces the ORT session load's file handling; ZASR_ERR_NOT_FOUND when files are missing. */
int zasr_convert_model(const char* model_dir, const char* out_dir);

/* Host-only (no GPU): the same for the single-graph models of the other stages, kind
   "silero" | "campp" | "vibert": read the file the reference opens in model_dir
   (silero_vad_16k_op15.onnx or silero_vad.onnx, core/vad_utils.py:22-24;
   campplus_cn_en_common_200k.onnx, core/speaker_diarization_senko_campp_optimized.py:324-325;
   vibert-capu.onnx or vibert-capu.int8.onnx, core/gec_model.py:133-140) -- or the engine's
   own <kind>_config.json + safetensors when present -- and write out_dir/<kind>_config.json +
   out_dir/{silero_vad,campp,vibert}.safetensors (torch state-dict names; the LSTM gates of
   the ONNX LSTM node reordered to torch's; a BatchNorm the exporter fused into its Conv kept
   as "<bn>.fused_shift").  zasr_vad_create / zasr_campp_create / zasr_vibert_create accept
   the reference's directories directly through the same reader. */
int zasr_convert_stage_model(const char* kind, const char* model_dir, const char* out_dir);

/* log-mel fbank of one waveform (f32 in [-1,1], 16 kHz).  out holds cap floats;
   *n_frames = (n + 80) / 160, output row-major [n_frames][80].  h may be NULL
   (uses device 0). */
int zasr_fbank(zasr_recognizer* h, const float* wav, int64_t n, int32_t sample_rate, float* out,
               int64_t cap, int64_t* n_frames);

/* The chunk planner's silence detector (core/asr_engine.py:521-554 find_silent_regions):
   for each of the n / frame_len frames of the HBM-resident signal d_wav (16-byte aligned),
   d_flags[f] = 1 when sqrt(mean(frame ** 2)) < threshold, evaluated exactly as numpy does
   in float32 (pairwise row sum, f32 divide, correctly rounded sqrt, f32 compare), else 0.
   frame_len: a multiple of 4, at most 256 (160 at 16 kHz).  Runs on `stream` (a hipStream_t,
   NULL = the default stream); needs no recognizer handle. */
int zasr_silence_flags(const float* d_wav, int64_t n, int32_t frame_len, float threshold,
                       uint8_t* d_flags, void* stream);

/* Decode `count` independent chunks (host buffers).  beam <= 0 uses the handle's
   configured decoding method / max_active_paths. */
int zasr_decode_batch(zasr_recognizer* h, const float* const* wav, const int64_t* n,
                      int32_t count, int32_t beam, zasr_result** out);

/* Same, from precomputed fbank features feats[i] of shape [n_frames[i]][80]. */
int zasr_decode_features(zasr_recognizer* h, const float* const* feats, const int64_t* n_frames,
                         int32_t count, int32_t beam, zasr_result** out);

/* Device-resident variant (inputs already in HBM): d_wav holds all chunks packed,
   chunk i at element offset wav_off[i] with n[i] samples (host arrays).  stream is a
   hipStream_t (NULL: the handle's stream).  Used by bench.py. */
int zasr_decode_device(zasr_recognizer* h, const float* d_wav, const int64_t* wav_off,
                       const int64_t* n, int32_t count, int32_t beam, void* stream,
                       zasr_result** out);

/* Several device-resident batches back to back: chunks as in zasr_decode_device, grouped
   into n_batches consecutive batches of batch_sizes[i] chunks (sum = count).  Batch k+1's
   fbank + encoder overlap batch k's search on the GPU; results for all count chunks, in
   chunk order, identical to decoding each batch with zasr_decode_device.  Replaces the
   reference's 2-worker chunk dispatch, whose point is that one worker's beam search runs
   while the other's encoder does (core/asr_engine.py:2250-2276). */
int zasr_decode_device_batches(zasr_recognizer* h, const float* d_wav, const int64_t* wav_off,
                               const int64_t* n, int32_t count, const int32_t* batch_sizes,
                               int32_t n_batches, int32_t beam, void* stream, zasr_result** out);

/* zasr_decode_device_batches from HOST waveforms (wav: host memory, pinned for an
   asynchronous copy, e.g. hipHostMalloc / torch pin_memory): each batch's span of samples is
   copied into the engine's device buffer for that pipeline slot on its own copy stream, and
   the batch's fbank waits for that copy alone, so batch k+1's upload runs under batch k's
   encoder and search.  Results identical to uploading the signal and calling
   zasr_decode_device_batches.  The reference's unit of work starts from the host waveform
   (core/asr_engine.py:2068). */
int zasr_decode_host_batches(zasr_recognizer* h, const float* wav, const int64_t* wav_off,
                             const int64_t* n, int32_t count, const int32_t* batch_sizes,
                             int32_t n_batches, int32_t beam, void* stream, zasr_result** out);

/* Encoder only: features -> encoder_out rows [T'_i][joiner_dim], packed in chunk order
   into out (cap floats); t_out[i] receives T'_i. */
int zasr_encode_features(zasr_recognizer* h, const float* const* feats, const int64_t* n_frames,
                         int32_t count, float* out, int64_t cap, int64_t* t_out);

/* Search only, from given encoder outputs enc[i] of shape [t_out[i]][joiner_dim]. */
int zasr_search_encoder_out(zasr_recognizer* h, const float* const* enc, const int64_t* t_out,
                            int32_t count, int32_t beam, zasr_result** out);

/* result access */
int32_t zasr_result_count(const zasr_result* r);
int32_t zasr_result_num_tokens(const zasr_result* r, int32_t i);
int32_t zasr_result_num_frames(const zasr_result* r, int32_t i); /* T' of chunk i */
const int32_t* zasr_result_tokens(const zasr_result* r, int32_t i);
const int32_t* zasr_result_frames(const zasr_result* r, int32_t i);
const double* zasr_result_log_probs(const zasr_result* r, int32_t i);
/* per token 4 floats: entropy, sum p^(1/3), top1 prob, top2 prob of the emitting row */
const float* zasr_result_token_stats(const zasr_result* r, int32_t i);
void zasr_result_free(zasr_result* r);

/* ---- offline streams: the sherpa-onnx OfflineRecognizer / OfflineStream surface ----
   The stream-shaped calls the reference's other callers bind: sherpa-onnx's C API
   (offline_pwa/static/vendor/sherpa-onnx-wasm/sherpa-onnx-asr.js:1782-1880) and its Python
   OfflineRecognizer (streaming_asr.py:224-243, core/audio_analyzer.py:345-361:
   create_stream -> accept_waveform -> decode_stream -> stream.result).  A stream holds host
   samples until decoded; zasr_decode_streams decodes several in ONE batched GPU pass (the
   zasr_decode_batch path), with the recognizer's configured method and beam.  A stream with
   fewer than 1360 samples (under 9 fbank frames) decodes to an empty result.
     zasr_create_stream            SherpaOnnxCreateOfflineStream (sherpa-onnx-asr.js:1862)
     zasr_destroy_stream           SherpaOnnxDestroyOfflineStream (:1790)
     zasr_stream_accept_waveform   SherpaOnnxAcceptWaveformOffline (:1799-1805); 16 kHz only
                                   (the reference resamples on load); appends
     zasr_decode_stream            SherpaOnnxDecodeOfflineStream (:1866-1868)
     zasr_decode_streams           SherpaOnnxDecodeMultipleOfflineStreams (one batch)
     zasr_stream_result_json       SherpaOnnxGetOfflineStreamResultAsJson (:1870-1878): keys
                                   lang, emotion, event, text, timestamps (frame x 0.04 s),
                                   tokens (tokens.txt strings, a leading U+2581 as a space, as
                                   sherpa-onnx's SymbolTable), ys_log_probs, words; *needed =
                                   bytes incl. the NUL (call with buf NULL to size it)
     zasr_stream_tokens / _frames / _log_probs / _token_stats / _num_*: the result arrays, as
                                   zasr_result_* for one chunk (valid until the stream is
                                   destroyed) */
typedef struct zasr_stream zasr_stream;
/* the symbol table zasr_stream_result_json's "tokens" / "text" use: sherpa-onnx's
   OfflineModelConfig.tokens (sherpa-onnx-asr.js:1719 tokens field; the reference passes
   tokens.txt beside its model files, core/asr_engine.py:980-986).  Default: model_dir/tokens.txt.
   ZASR_ERR_NOT_FOUND if the file does not exist. */
int zasr_set_tokens(zasr_recognizer* h, const char* tokens_path);
int zasr_create_stream(zasr_recognizer* h, zasr_stream** out);
void zasr_destroy_stream(zasr_stream* s);
int zasr_stream_accept_waveform(zasr_stream* s, int32_t sample_rate, const float* samples,
                                int64_t n);
int zasr_decode_stream(zasr_recognizer* h, zasr_stream* s);
int zasr_decode_streams(zasr_recognizer* h, zasr_stream* const* streams, int32_t n);
int32_t zasr_stream_is_decoded(const zasr_stream* s);
int32_t zasr_stream_num_tokens(const zasr_stream* s);
int32_t zasr_stream_num_frames(const zasr_stream* s);
const int32_t* zasr_stream_tokens(const zasr_stream* s);
const int32_t* zasr_stream_frames(const zasr_stream* s);
const double* zasr_stream_log_probs(const zasr_stream* s);
const float* zasr_stream_token_stats(const zasr_stream* s);
int zasr_stream_result_json(const zasr_stream* s, char* buf, int64_t cap, int64_t* needed);

/* ---- CAM++ speaker embedding ----
   Replaces the reference's onnxruntime CAM++ session and its numpy front end:
   core/speaker_diarization_senko_campp_optimized.py:86-159 (_compute_fbank_vectorized),
   :589-605 (batched emb_sess.run(['embs'], {'feats': batch})); the model is the reference's
   convert_onnx/export_campplus_onnx.py CAMPPlus (192-dim).  model_dir holds the reference's
   campplus_cn_en_common_200k.onnx (Conv+BN fused by the exporter or not) or
   campp_config.json + campp.safetensors (state-dict names); see zasr_convert_stage_model. */
typedef struct zasr_campp zasr_campp;
int zasr_campp_create(const char* model_dir, int32_t device_id, zasr_campp** out);
void zasr_campp_destroy(zasr_campp* h);
int32_t zasr_campp_embedding_dim(const zasr_campp* h);
/* fbank + per-utterance CMVN of one waveform: *n_frames = 1 + (n - 400) / 160 (0 if n < 400) */
int zasr_campp_fbank(zasr_campp* h, const float* wav, int64_t n, float* out, int64_t cap,
                     int64_t* n_frames);
/* embeddings of a feature batch [count][n_frames][80] (zero-padded like the reference's
   batch tensor) -> out [count][embedding_dim] (not L2-normalised, as the ONNX output) */
int zasr_campp_embed(zasr_campp* h, const float* feats, int32_t count, int32_t n_frames,
                     float* out);
/* same with device buffers on `stream` (NULL: the handle's stream); used by bench.py */
int zasr_campp_embed_device(zasr_campp* h, const float* d_feats, int32_t count,
                            int32_t n_frames, float* d_out, void* stream);
/* the front end of a whole file in HBM: fbank + per-region CMVN of every speech region
   [region_off[i], + region_len[i]) of d_wav, then the windows of window_frames frames every
   step_frames (tail pulled back; a region shorter than a window gives one window of all its
   frames, zero-padded; < 10 frames: none) gathered into d_feats [n][window_frames][80] on
   `stream`.  Replaces _sliding_window_embeddings' fbank-once-slice-later loop and batch
   tensor (core/speaker_diarization_senko_campp_optimized.py:540-600).  *n_windows = n;
   window_region / window_first / window_nframes (host, capacity max_windows) describe each
   window (its start time is region start + first * 10 ms, :567-577). */
int zasr_campp_windows_device(zasr_campp* h, const float* d_wav, const int64_t* region_off,
                              const int64_t* region_len, int32_t n_regions, int32_t window_frames,
                              int32_t step_frames, float* d_feats, int64_t max_windows,
                              int32_t* window_region, int32_t* window_first,
                              int32_t* window_nframes, int64_t* n_windows, void* stream);

/* ---- ViBERT-capu punctuation / capitalization ----
   Replaces the reference's onnxruntime session of vibert-capu.onnx (core/gec_model.py:
   366-412: session.run(None, {input_ids, attention_mask, token_type_ids, input_offsets}) ->
   (logits, detect_logits)); graph: convert_onnx/export_vibert_onnx.py Seq2LabelsModel.
   model_dir holds the reference's vibert-capu.onnx (or .int8.onnx, dequantized; config.json
   beside it gives the head count, else head dim 64) or vibert_config.json +
   vibert.safetensors (Hugging Face names); see zasr_convert_stage_model. */
typedef struct zasr_vibert zasr_vibert;
int zasr_vibert_create(const char* model_dir, int32_t device_id, zasr_vibert** out);
void zasr_vibert_destroy(zasr_vibert* h);
int32_t zasr_vibert_num_labels(const zasr_vibert* h);
int32_t zasr_vibert_num_detect(const zasr_vibert* h);
/* inputs int64 [batch][n_tokens] (ids, mask, token types) and [batch][n_words] offsets;
   outputs logits [batch][n_words][num_labels], detect_logits [batch][n_words][num_detect] */
int zasr_vibert_run(zasr_vibert* h, const int64_t* input_ids, const int64_t* attention_mask,
                    const int64_t* token_type_ids, const int64_t* input_offsets, int32_t batch,
                    int32_t n_tokens, int32_t n_words, float* logits, float* detect_logits);

/* ---- Silero VAD ----
   Replaces the reference's per-window onnxruntime loop over silero_vad_16k_op15.onnx
   (core/vad_utils.py:62-111: 64-sample context + 512-sample window, (2, 1, 128) LSTM state
   carried across calls).  model_dir holds the reference's silero_vad_16k_op15.onnx (or
   silero_vad.onnx; the 16 kHz branch is found by walking the graph, If branches included) or
   silero_config.json + silero_vad.safetensors (torch state-dict names of the 16 kHz model);
   see zasr_convert_stage_model. */
typedef struct zasr_vad zasr_vad;
int zasr_vad_create(const char* model_dir, int32_t device_id, zasr_vad** out);
void zasr_vad_destroy(zasr_vad* h);
/* speech probability of every full 512-sample window of n_files files (file i = audio
   [offsets[i], offsets[i] + lengths[i])), state reset per file as in _run_vad_inference;
   probs of file i start at sum_{k<i} lengths[k] / 512.  auto_boost != 0 scales a file whose
   peak is in (1e-6, 0.071) to a 0.071 peak first (get_vad_segments, vad_utils.py:203-208).
   Host buffers. */
int zasr_vad_probs(zasr_vad* h, const float* audio, const int64_t* offsets,
                   const int64_t* lengths, int32_t n_files, int32_t auto_boost, float* probs);
/* the same with device-resident audio and probs; ordered after / before `stream`
   (a hipStream_t, 0 = synchronous) */
int zasr_vad_probs_device(zasr_vad* h, const float* d_audio, const int64_t* offsets,
                          const int64_t* lengths, int32_t n_files, int32_t auto_boost,
                          float* d_probs, void* stream);
/* recurrence passes of the last probs call: a long file is decoded as parallel segments whose
   chained start states are checked against their predecessors' end states to a relative
   1e-6 per element (the rounding-noise level of two summation orders; NOT bit-exact: the
   probabilities stay within ~2.4e-7 of the sequential recurrence and give the same speech
   segments, tests/test_gpu_vad.py).  1 = every warm-up guess passed; set ZASR_VAD_PIT=0
   before create for one sequential workgroup per file */
int32_t zasr_vad_last_passes(const zasr_vad* h);
/* one session.run step for n independent streams: input [n][576], state [2][n][128] ->
   prob [n], state_out [2][n][128] (the ORT session surface, vad_utils.py:100-102) */
int zasr_vad_window(zasr_vad* h, const float* input, const float* state, int32_t n, float* prob,
                    float* state_out);

/* model facts */
int32_t zasr_vocab_size(const zasr_recognizer* h);
int32_t zasr_joiner_dim(const zasr_recognizer* h);
/* which kernel each part of the loaded model was routed to, as JSON into buf (cap bytes):
   {"precision", "ffn_fused_h3", "ffn_gemm_pair", "gemm_h3r", "gemm_x3_range", "cnx_ffn_h3",
   "dec_table"}.  In f16x3 a layer whose weights reach 31 in magnitude keeps the
   two-accumulator GEMMs (the one-accumulator kernels scale the weight's fp16 hi piece by
   2^11); a vocabulary whose V^2 x D decoder-context table exceeds ZASR_DEC_TABLE_MAX_GB
   (default 24) runs the per-frame decoder instead (dec_table 0).  No reference counterpart:
   a diagnostic of this build's dispatch, read by the tests. */
int zasr_model_routes(zasr_recognizer* h, char* buf, int64_t cap);
/* Replace the fbank's 80 triangular filters: banks row-major [80][n_bins] (n_bins 256, or
   257 with the Nyquist column zero).  The default is knf's mel-linear triangles
   (core/asr_engine.py:698-721); the reference's browser worker computes Hz-linear triangles
   (offline_pwa/static/js/pure-ort-asr-worker.js:369-397), which lets a test hold this kernel
   to that worker's own outputs.  Applies to later zasr_fbank / decode calls on h. */
int zasr_fbank_set_mel_banks(zasr_recognizer* h, const float* banks, int32_t n_bins);
/* Launch a no-op kernel with block_threads threads per block through the library's checked
   launch path (every kernel launch is followed by the runtime's launch status): a refused
   configuration (e.g. > 1024 threads) returns ZASR_ERR_RUNTIME with the HIP error in
   zasr_last_error().  No reference counterpart: a self-test of the error path. */
int zasr_selftest_launch(int32_t block_threads);
/* Kernel self-tests of the f16x3 one-accumulator kernels on host operands (device 0,
   synchronous; no reference counterpart: test infrastructure that reaches the shapes and row
   counts the decode meets only incidentally).  gemm_h3r: C[M][N'] = epi(A[M][K] W[N][K]^T +
   bias), epi 0 (none), 3 (C += ..., C is read) or 8 (GLU over interleaved rows, N' = N / 2);
   K in {96, 192, 256, 288, 384, 512}, N >= 128, N % 16 == 0.  ffn_h3: X[R][D] += W2
   SwooshL(W1 Y + b1) + b2, then X = byp_orig + (X - byp_orig) * byp_scale when byp_orig is
   given (the bypass_mid epilogue); D in {128, 256, 384, 512} (F % 32 == 0) or 192
   (F % 64 == 0).  Every |w| must be below 31 (the kernels scale the fp16 hi piece by 2^11). */
int zasr_selftest_gemm_h3r(int32_t M, int32_t K, int32_t N, int32_t epi, const float* A,
                           const float* W, const float* bias, float* C);
int zasr_selftest_ffn_h3(int32_t R, int32_t D, int32_t F, const float* Y, const float* W1,
                         const float* b1, const float* W2, const float* b2,
                         const float* byp_orig, const float* byp_scale, float* X);
/* The bf16 mode's fused FeedforwardModule alone on host operands (same conventions):
   X[R][D] += W2 SwooshL(W1 bf16(X) + b1) + b2 with W1 [F][D], W2 [D][F] rounded to bf16 and
   the hidden activation in bf16 (then the bypass_mid blend when byp_orig is given);
   D in {64, 96, 128, 192, 256, 384, 512}; D >= 256: F % 32 == 0, F <= 2048.  form 0: the
   decode's route; 1: the opt-in per-CU rows form at D = 384 (ZASR_FFN_ROWS=1). */
int zasr_selftest_ffn_bf16(int32_t R, int32_t D, int32_t F, const float* W1, const float* b1,
                           const float* W2, const float* b2, const float* byp_orig,
                           const float* byp_scale, float* X, int32_t form);

/* profiling: per-kernel-class HIP-event timing on the handle's stream.  on = 0 off,
   1 kernel classes, 2 kernel classes with the encoder GEMMs split by shape
   ("enc_gemm|M|K|N|w16|a16|c16|epi" class names, for the per-shape roofline table) */
int zasr_profile_enable(zasr_recognizer* h, int32_t on);
int zasr_profile_reset(zasr_recognizer* h);
/* writes "name count total_ms\n" lines into buf (cap bytes) */
int zasr_profile_report(zasr_recognizer* h, char* buf, int64_t cap);

const char* zasr_last_error(void);
const char* zasr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ZASR_H_ */
