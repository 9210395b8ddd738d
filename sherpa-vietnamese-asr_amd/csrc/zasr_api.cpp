// C ABI of libzasr (include/zasr.h): argument checking, error capture, result objects.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/zasr.h"
#include "campp.h"
#include "common.h"
#include "vad.h"
#include "vibert.h"
#include "engine.h"
#include "host_io.h"
#include "onnx_io.h"

using zasr::Engine;
using zasr::TokenResult;

struct zasr_recognizer {
  std::unique_ptr<Engine> eng;
  std::string model_dir;
  // the symbol table (sherpa-onnx OfflineModelConfig.tokens; zasr_set_tokens, default
  // model_dir/tokens.txt), loaded on the first JSON result (sherpa-onnx SymbolTable: a
  // leading "\u2581" becomes a space)
  std::string tokens_path;
  std::mutex sym_mu;
  // immutable once published: a reader copies the pointer under sym_mu and keeps its table
  // alive across a concurrent zasr_set_tokens, which only swaps the pointer
  std::shared_ptr<const std::vector<std::string>> syms;
};

// an offline stream (sherpa-onnx OfflineStream): the samples accepted so far and, once
// decoded, its result; bound to the recognizer that created it
struct zasr_stream {
  zasr_recognizer* rec = nullptr;
  std::vector<float> samples;
  bool decoded = false;
  TokenResult res;
};

struct zasr_result {
  std::vector<TokenResult> items;
};

struct zasr_campp {
  std::unique_ptr<zasr::CamppEngine> eng;
};

struct zasr_vibert {
  std::unique_ptr<zasr::VibertEngine> eng;
};

struct zasr_vad {
  std::unique_ptr<zasr::VadEngine> eng;
};

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::invalid_argument& e) {
    return fail(ZASR_ERR_NOT_FOUND, e.what());
  } catch (const std::exception& e) {
    return fail(ZASR_ERR_RUNTIME, e.what());
  } catch (...) {
    return fail(ZASR_ERR_RUNTIME, "unknown error");
  }
}

int resolve_beam(zasr_recognizer* h, int32_t beam) {
  return beam > 0 ? beam : h->eng->default_beam();
}

// fewest samples the encoder accepts: 9 fbank frames ((n + 80) / 160 >= 9); shorter streams
// decode to an empty result, as an encoder output of no frames does
constexpr long kMinStreamSamples = 9 * 160 - 80;

// Decode streams [s0, s1, ...] of one recognizer in ONE batched pass (host samples staged
// into one device buffer, the zasr_decode_batch path); results stored in the streams.
void decode_streams_impl(zasr_recognizer* h, zasr_stream* const* ss, int n) {
  Engine* e = h->eng.get();
  std::vector<int> idx;
  std::vector<long> off, len;
  long tot = 0;
  for (int i = 0; i < n; ++i) {
    const long m = (long)ss[i]->samples.size();
    if (m < kMinStreamSamples) {
      ss[i]->res = TokenResult{};
      ss[i]->decoded = true;
      continue;
    }
    idx.push_back(i);
    off.push_back(tot);
    len.push_back(m);
    tot += m;
  }
  if (idx.empty()) return;
  std::lock_guard<std::mutex> lk(e->mu);
  float* d = nullptr;
  ZASR_HIP_CHECK(hipMalloc(&d, tot * sizeof(float)));
  std::unique_ptr<float, decltype(&hipFree)> guard(d, hipFree);
  for (size_t j = 0; j < idx.size(); ++j)
    ZASR_HIP_CHECK(hipMemcpyAsync(d + off[j], ss[idx[j]]->samples.data(), len[j] * 4,
                                  hipMemcpyHostToDevice, e->stream()));
  std::vector<TokenResult> r = e->decode_device(d, off, len, e->default_beam(), e->stream());
  ZASR_HIP_CHECK(hipStreamSynchronize(e->stream()));
  for (size_t j = 0; j < idx.size(); ++j) {
    ss[idx[j]]->res = std::move(r[j]);
    ss[idx[j]]->decoded = true;
  }
}

std::shared_ptr<const std::vector<std::string>> symbols(zasr_recognizer* h) {
  std::lock_guard<std::mutex> lk(h->sym_mu);
  if (!h->syms) {
    const std::string path = h->tokens_path.empty() ? h->model_dir + "/tokens.txt" : h->tokens_path;
    std::ifstream f(path);
    if (!f) throw std::invalid_argument("symbol table not found: " + path);
    auto tab = std::make_shared<std::vector<std::string>>();
    std::string line;
    while (std::getline(f, line)) {
      std::istringstream ls(line);
      std::string sym, id_s;
      if (!(ls >> sym >> id_s)) continue;
      const long id = std::stol(id_s);
      if (id < 0) continue;
      if (sym.compare(0, 3, "\xe2\x96\x81") == 0) sym.replace(0, 3, " ");
      if ((long)tab->size() <= id) tab->resize(id + 1);
      (*tab)[id] = sym;
    }
    h->syms = std::move(tab);
  }
  return h->syms;
}

void json_string(std::ostringstream& os, const std::string& s) {
  os << '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') os << '\\' << c;
    else if (c < 0x20) {
      char b[8];
      std::snprintf(b, sizeof b, "\\u%04x", c);
      os << b;
    } else os << c;
  }
  os << '"';
}

}  // namespace

extern "C" {

int zasr_create(const zasr_config* cfg, zasr_recognizer** out) {
  if (!cfg || !out || !cfg->model_dir) return fail(ZASR_ERR_INVALID, "null config/model_dir/out");
  *out = nullptr;
  if (cfg->blank_penalty != 0.f) return fail(ZASR_ERR_INVALID, "blank_penalty must be 0");
  std::string method = cfg->decoding_method ? cfg->decoding_method : "modified_beam_search";
  bool greedy = (method == "greedy_search");
  if (!greedy && method != "modified_beam_search")
    return fail(ZASR_ERR_INVALID, "decoding_method must be greedy_search or modified_beam_search");
  int beam = greedy ? 1 : cfg->max_active_paths;
  if (beam < 1 || beam > 16) return fail(ZASR_ERR_INVALID, "max_active_paths must be in 1..16");
  if (cfg->num_hotwords < 0) return fail(ZASR_ERR_INVALID, "num_hotwords < 0");
  return guarded([&]() {
    std::vector<std::vector<int>> phrases;
    std::vector<float> scores;
    const int32_t* tp = cfg->hotword_tokens;
    for (int i = 0; i < cfg->num_hotwords; ++i) {
      int n = cfg->hotword_lens[i];
      if (n < 0) return fail(ZASR_ERR_INVALID, "negative hotword length");
      phrases.emplace_back(tp, tp + n);
      tp += n;
      scores.push_back(cfg->hotword_scores[i]);
    }
    auto* h = new zasr_recognizer;
    try {
      h->eng.reset(new Engine(cfg->model_dir, cfg->device_id, beam, greedy, phrases, scores,
                              cfg->precision));
    } catch (...) {
      delete h;
      throw;
    }
    h->model_dir = cfg->model_dir;
    *out = h;
    return (int)ZASR_OK;
  });
}

void zasr_destroy(zasr_recognizer* h) { delete h; }

int zasr_campp_create(const char* model_dir, int32_t device_id, zasr_campp** out) {
  if (!model_dir || !out) return fail(ZASR_ERR_INVALID, "null model_dir/out");
  *out = nullptr;
  return guarded([&]() {
    auto* h = new zasr_campp;
    try {
      h->eng.reset(new zasr::CamppEngine(model_dir, device_id));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
    return (int)ZASR_OK;
  });
}

void zasr_campp_destroy(zasr_campp* h) { delete h; }

int32_t zasr_campp_embedding_dim(const zasr_campp* h) { return h ? h->eng->emb_dim() : 0; }

int zasr_vibert_create(const char* model_dir, int32_t device_id, zasr_vibert** out) {
  if (!model_dir || !out) return fail(ZASR_ERR_INVALID, "null model_dir/out");
  *out = nullptr;
  return guarded([&]() {
    auto* h = new zasr_vibert;
    try {
      h->eng.reset(new zasr::VibertEngine(model_dir, device_id));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
    return (int)ZASR_OK;
  });
}

void zasr_vibert_destroy(zasr_vibert* h) { delete h; }

int32_t zasr_vibert_num_labels(const zasr_vibert* h) { return h ? h->eng->num_labels() : 0; }
int32_t zasr_vibert_num_detect(const zasr_vibert* h) { return h ? h->eng->num_detect() : 0; }

int zasr_vibert_run(zasr_vibert* h, const int64_t* input_ids, const int64_t* attention_mask,
                    const int64_t* token_type_ids, const int64_t* input_offsets, int32_t batch,
                    int32_t n_tokens, int32_t n_words, float* logits, float* detect_logits) {
  if (!h || (batch > 0 && (!input_ids || !attention_mask || !token_type_ids || !input_offsets ||
                           !logits || !detect_logits)))
    return fail(ZASR_ERR_INVALID, "null argument");
  if (batch < 0 || n_tokens < 1 || n_words < 1) return fail(ZASR_ERR_INVALID, "bad batch shape");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->run_host(reinterpret_cast<const long*>(input_ids), reinterpret_cast<const long*>(attention_mask),
                     reinterpret_cast<const long*>(token_type_ids),
                     reinterpret_cast<const long*>(input_offsets), batch, n_tokens, n_words, logits,
                     detect_logits);
    return (int)ZASR_OK;
  });
}

int zasr_vad_create(const char* model_dir, int32_t device_id, zasr_vad** out) {
  if (!model_dir || !out) return fail(ZASR_ERR_INVALID, "null model_dir/out");
  *out = nullptr;
  return guarded([&]() {
    auto* h = new zasr_vad;
    try {
      h->eng.reset(new zasr::VadEngine(model_dir, device_id));
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
    return (int)ZASR_OK;
  });
}

void zasr_vad_destroy(zasr_vad* h) { delete h; }

int32_t zasr_vad_last_passes(const zasr_vad* h) { return h ? h->eng->last_passes() : 0; }

int zasr_vad_probs(zasr_vad* h, const float* audio, const int64_t* offsets,
                   const int64_t* lengths, int32_t n_files, int32_t auto_boost, float* probs) {
  if (!h || n_files < 0 || (n_files > 0 && (!audio || !offsets || !lengths || !probs)))
    return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->probs_host(audio, reinterpret_cast<const long*>(offsets),
                       reinterpret_cast<const long*>(lengths), n_files, auto_boost != 0, probs);
    return (int)ZASR_OK;
  });
}

int zasr_vad_probs_device(zasr_vad* h, const float* d_audio, const int64_t* offsets,
                          const int64_t* lengths, int32_t n_files, int32_t auto_boost,
                          float* d_probs, void* stream) {
  if (!h || n_files < 0 || (n_files > 0 && (!d_audio || !offsets || !lengths || !d_probs)))
    return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->probs_device(d_audio, reinterpret_cast<const long*>(offsets),
                         reinterpret_cast<const long*>(lengths), n_files, auto_boost != 0, d_probs,
                         reinterpret_cast<hipStream_t>(stream));
    return (int)ZASR_OK;
  });
}

int zasr_vad_window(zasr_vad* h, const float* input, const float* state, int32_t n, float* prob,
                    float* state_out) {
  if (!h || n < 0 || (n > 0 && (!input || !state || !prob || !state_out)))
    return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->window_host(input, state, n, prob, state_out);
    return (int)ZASR_OK;
  });
}

int zasr_campp_fbank(zasr_campp* h, const float* wav, int64_t n, float* out, int64_t cap,
                     int64_t* n_frames) {
  if (!h || !n_frames || (n > 0 && !wav)) return fail(ZASR_ERR_INVALID, "null argument");
  const int64_t frames = n >= 400 ? 1 + (n - 400) / 160 : 0;
  *n_frames = frames;
  if (frames * 80 > cap || (frames > 0 && !out)) return fail(ZASR_ERR_INVALID, "output buffer too small");
  if (frames == 0) return ZASR_OK;
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    std::vector<float> f;
    h->eng->fbank_host(wav, (long)n, f);
    std::memcpy(out, f.data(), f.size() * sizeof(float));
    return (int)ZASR_OK;
  });
}

int zasr_campp_embed(zasr_campp* h, const float* feats, int32_t count, int32_t n_frames,
                     float* out) {
  if (!h || (count > 0 && (!feats || !out))) return fail(ZASR_ERR_INVALID, "null argument");
  if (count < 0 || n_frames < 1) return fail(ZASR_ERR_INVALID, "count >= 0 and n_frames >= 1 required");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->embed_host(feats, count, n_frames, out);
    return (int)ZASR_OK;
  });
}

int zasr_campp_embed_device(zasr_campp* h, const float* d_feats, int32_t count, int32_t n_frames,
                            float* d_out, void* stream) {
  if (!h || (count > 0 && (!d_feats || !d_out))) return fail(ZASR_ERR_INVALID, "null argument");
  if (count < 0 || n_frames < 1) return fail(ZASR_ERR_INVALID, "count >= 0 and n_frames >= 1 required");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->embed_device(d_feats, count, n_frames, d_out, reinterpret_cast<hipStream_t>(stream));
    return (int)ZASR_OK;
  });
}

int zasr_campp_windows_device(zasr_campp* h, const float* d_wav, const int64_t* region_off,
                              const int64_t* region_len, int32_t n_regions, int32_t window_frames,
                              int32_t step_frames, float* d_feats, int64_t max_windows,
                              int32_t* window_region, int32_t* window_first,
                              int32_t* window_nframes, int64_t* n_windows, void* stream) {
  if (!h || !n_windows || n_regions < 0 || (n_regions > 0 && (!d_wav || !region_off || !region_len)) ||
      max_windows < 0 || (max_windows > 0 && (!d_feats || !window_region || !window_first || !window_nframes)))
    return fail(ZASR_ERR_INVALID, "null argument");
  if (window_frames < 1 || step_frames < 1)
    return fail(ZASR_ERR_INVALID, "window_frames and step_frames must be >= 1");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    *n_windows = h->eng->windows_device(d_wav, reinterpret_cast<const long*>(region_off),
                                        reinterpret_cast<const long*>(region_len), n_regions,
                                        window_frames, step_frames, d_feats, max_windows,
                                        window_region, window_first, window_nframes,
                                        reinterpret_cast<hipStream_t>(stream));
    return (int)ZASR_OK;
  });
}

int zasr_convert_model(const char* model_dir, const char* out_dir) {
  if (!model_dir || !out_dir) return fail(ZASR_ERR_INVALID, "null model_dir/out_dir");
  return guarded([&]() {
    zasr::SafeTensors w;
    const std::string cfg = zasr::load_model_dir(model_dir, w);
    zasr::write_safetensors(std::string(out_dir) + "/model.safetensors", w);
    FILE* f = fopen((std::string(out_dir) + "/config.json").c_str(), "wb");
    if (!f) return fail(ZASR_ERR_RUNTIME, std::string("cannot write config.json in ") + out_dir);
    const size_t wr = fwrite(cfg.data(), 1, cfg.size(), f);
    fclose(f);
    if (wr != cfg.size()) return fail(ZASR_ERR_RUNTIME, "short write of config.json");
    return (int)ZASR_OK;
  });
}

int zasr_convert_stage_model(const char* kind, const char* model_dir, const char* out_dir) {
  if (!kind || !model_dir || !out_dir) return fail(ZASR_ERR_INVALID, "null kind/model_dir/out_dir");
  const std::string k(kind);
  if (k != "silero" && k != "campp" && k != "vibert")
    return fail(ZASR_ERR_INVALID, "kind must be silero, campp or vibert");
  return guarded([&]() {
    zasr::SafeTensors w;
    const std::string cfg = zasr::load_stage_dir(model_dir, k, w);
    zasr::write_safetensors(std::string(out_dir) + "/" + zasr::stage_safetensors_name(k), w);
    const std::string cp = std::string(out_dir) + "/" + k + "_config.json";
    FILE* f = fopen(cp.c_str(), "wb");
    if (!f) return fail(ZASR_ERR_RUNTIME, "cannot write " + cp);
    const size_t wr = fwrite(cfg.data(), 1, cfg.size(), f);
    fclose(f);
    if (wr != cfg.size()) return fail(ZASR_ERR_RUNTIME, "short write of " + cp);
    return (int)ZASR_OK;
  });
}

int zasr_fbank(zasr_recognizer* h, const float* wav, int64_t n, int32_t sr, float* out,
               int64_t cap, int64_t* n_frames) {
  if (!n_frames || (n > 0 && !wav)) return fail(ZASR_ERR_INVALID, "null argument");
  if (sr != 16000) return fail(ZASR_ERR_INVALID, "sample rate must be 16000");
  int64_t frames = n > 0 ? (n + 80) / 160 : 0;
  *n_frames = frames;
  if (frames * 80 > cap || (frames > 0 && !out)) return fail(ZASR_ERR_INVALID, "output buffer too small");
  if (frames == 0) return ZASR_OK;
  return guarded([&]() {
    Engine* e = h ? h->eng.get() : nullptr;
    if (!e) return fail(ZASR_ERR_INVALID, "zasr_fbank needs a recognizer handle");
    std::lock_guard<std::mutex> lk(e->mu);
    e->fbank_host(wav, (long)n, out);
    return (int)ZASR_OK;
  });
}

int zasr_decode_batch(zasr_recognizer* h, const float* const* wav, const int64_t* n,
                      int32_t count, int32_t beam, zasr_result** out) {
  if (!h || !out || count < 0 || (count > 0 && (!wav || !n))) return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    // stage host chunks into one device buffer, then run the device path
    std::vector<long> off(count), len(count);
    long tot = 0;
    for (int i = 0; i < count; ++i) {
      if (n[i] < 0) return fail(ZASR_ERR_INVALID, "negative length");
      off[i] = tot;
      len[i] = (long)n[i];
      tot += (long)n[i];
    }
    float* d = nullptr;
    ZASR_HIP_CHECK(hipMalloc(&d, std::max<long>(tot, 1) * sizeof(float)));
    std::unique_ptr<float, decltype(&hipFree)> guard(d, hipFree);
    for (int i = 0; i < count; ++i)
      if (len[i] > 0)
        ZASR_HIP_CHECK(hipMemcpyAsync(d + off[i], wav[i], len[i] * 4, hipMemcpyHostToDevice, e->stream()));
    auto r = std::make_unique<zasr_result>();
    r->items = e->decode_device(d, off, len, resolve_beam(h, beam), e->stream());
    ZASR_HIP_CHECK(hipStreamSynchronize(e->stream()));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int zasr_decode_features(zasr_recognizer* h, const float* const* feats, const int64_t* n_frames,
                         int32_t count, int32_t beam, zasr_result** out) {
  if (!h || !out || count < 0 || (count > 0 && (!feats || !n_frames))) return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<const float*> f(feats, feats + count);
    std::vector<long> fr(n_frames, n_frames + count);
    auto r = std::make_unique<zasr_result>();
    r->items = e->decode_features(f, fr, resolve_beam(h, beam));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int zasr_decode_device(zasr_recognizer* h, const float* d_wav, const int64_t* wav_off,
                       const int64_t* n, int32_t count, int32_t beam, void* stream,
                       zasr_result** out) {
  if (!h || !out || count < 0 || (count > 0 && (!d_wav || !wav_off || !n))) return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<long> off(wav_off, wav_off + count), len(n, n + count);
    auto r = std::make_unique<zasr_result>();
    r->items = e->decode_device(d_wav, off, len, resolve_beam(h, beam),
                                reinterpret_cast<hipStream_t>(stream));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int zasr_decode_device_batches(zasr_recognizer* h, const float* d_wav, const int64_t* wav_off,
                               const int64_t* n, int32_t count, const int32_t* batch_sizes,
                               int32_t n_batches, int32_t beam, void* stream, zasr_result** out) {
  if (!h || !out || count < 0 || n_batches < 0 || (n_batches > 0 && !batch_sizes) ||
      (count > 0 && (!d_wav || !wav_off || !n)))
    return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  long total = 0;
  for (int32_t i = 0; i < n_batches; ++i) {
    if (batch_sizes[i] < 0) return fail(ZASR_ERR_INVALID, "negative batch size");
    total += batch_sizes[i];
  }
  if (total != count) return fail(ZASR_ERR_INVALID, "batch sizes must sum to count");
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<long> off(wav_off, wav_off + count), len(n, n + count);
    std::vector<int> bs(batch_sizes, batch_sizes + n_batches);
    auto r = std::make_unique<zasr_result>();
    r->items = e->decode_device_batches(d_wav, off, len, bs, resolve_beam(h, beam),
                                        reinterpret_cast<hipStream_t>(stream));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int zasr_decode_host_batches(zasr_recognizer* h, const float* wav, const int64_t* wav_off,
                             const int64_t* n, int32_t count, const int32_t* batch_sizes,
                             int32_t n_batches, int32_t beam, void* stream, zasr_result** out) {
  if (!h || !out || count < 0 || n_batches < 0 || (n_batches > 0 && !batch_sizes) ||
      (count > 0 && (!wav || !wav_off || !n)))
    return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  long total = 0;
  for (int32_t i = 0; i < n_batches; ++i) {
    if (batch_sizes[i] < 0) return fail(ZASR_ERR_INVALID, "negative batch size");
    total += batch_sizes[i];
  }
  if (total != count) return fail(ZASR_ERR_INVALID, "batch sizes must sum to count");
  for (int32_t i = 0; i < count; ++i)
    if (wav_off[i] < 0 || n[i] < 0) return fail(ZASR_ERR_INVALID, "negative offset or length");
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<long> off(wav_off, wav_off + count), len(n, n + count);
    std::vector<int> bs(batch_sizes, batch_sizes + n_batches);
    auto r = std::make_unique<zasr_result>();
    r->items = e->decode_host_batches(wav, off, len, bs, resolve_beam(h, beam),
                                      reinterpret_cast<hipStream_t>(stream));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int zasr_encode_features(zasr_recognizer* h, const float* const* feats, const int64_t* n_frames,
                         int32_t count, float* out, int64_t cap, int64_t* t_out) {
  if (!h || !feats || !n_frames || !out || !t_out || count <= 0) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<const float*> f(feats, feats + count);
    std::vector<long> fr(n_frames, n_frames + count);
    long need = 0;
    for (int i = 0; i < count; ++i) {
      if (n_frames[i] < 9) return fail(ZASR_ERR_INVALID, "chunk shorter than 9 fbank frames");
      need += ((n_frames[i] - 7) / 2 + 1) / 2;
    }
    if (need * e->joiner_dim() > cap) return fail(ZASR_ERR_INVALID, "output buffer too small");
    std::vector<float> enc;
    std::vector<int> to;
    e->encode_host(f, fr, enc, to);
    std::memcpy(out, enc.data(), enc.size() * sizeof(float));
    for (int i = 0; i < count; ++i) t_out[i] = to[i];
    return (int)ZASR_OK;
  });
}

int zasr_search_encoder_out(zasr_recognizer* h, const float* const* enc, const int64_t* t_out,
                            int32_t count, int32_t beam, zasr_result** out) {
  if (!h || !enc || !t_out || !out || count < 0) return fail(ZASR_ERR_INVALID, "null argument");
  *out = nullptr;
  return guarded([&]() {
    Engine* e = h->eng.get();
    std::lock_guard<std::mutex> lk(e->mu);
    std::vector<const float*> p(enc, enc + count);
    std::vector<long> t(t_out, t_out + count);
    auto r = std::make_unique<zasr_result>();
    r->items = e->search_host(p, t, resolve_beam(h, beam));
    *out = r.release();
    return (int)ZASR_OK;
  });
}

int32_t zasr_result_count(const zasr_result* r) { return r ? (int32_t)r->items.size() : 0; }
static const TokenResult* item(const zasr_result* r, int32_t i) {
  return (r && i >= 0 && i < (int32_t)r->items.size()) ? &r->items[i] : nullptr;
}
int32_t zasr_result_num_tokens(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? (int32_t)t->tok.size() : 0;
}
int32_t zasr_result_num_frames(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? t->t_out : 0;
}
const int32_t* zasr_result_tokens(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? t->tok.data() : nullptr;
}
const int32_t* zasr_result_frames(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? t->frame.data() : nullptr;
}
const double* zasr_result_log_probs(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? t->lp.data() : nullptr;
}
const float* zasr_result_token_stats(const zasr_result* r, int32_t i) {
  auto* t = item(r, i);
  return t ? t->stats.data() : nullptr;
}
void zasr_result_free(zasr_result* r) { delete r; }

int32_t zasr_vocab_size(const zasr_recognizer* h) { return h ? h->eng->vocab() : 0; }
int32_t zasr_joiner_dim(const zasr_recognizer* h) { return h ? h->eng->joiner_dim() : 0; }

int zasr_profile_enable(zasr_recognizer* h, int32_t on) {
  if (!h) return fail(ZASR_ERR_INVALID, "null handle");
  if (on < 0 || on > 2) return fail(ZASR_ERR_INVALID, "profile mode must be 0, 1 or 2");
  h->eng->profile_enable((int)on);
  return ZASR_OK;
}
int zasr_profile_reset(zasr_recognizer* h) {
  if (!h) return fail(ZASR_ERR_INVALID, "null handle");
  return guarded([&]() {
    h->eng->profile_reset();
    return (int)ZASR_OK;
  });
}
int zasr_profile_report(zasr_recognizer* h, char* buf, int64_t cap) {
  if (!h || !buf || cap <= 0) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    std::string s = h->eng->profile_report();
    if ((int64_t)s.size() + 1 > cap) return fail(ZASR_ERR_INVALID, "report buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)ZASR_OK;
  });
}

int zasr_model_routes(zasr_recognizer* h, char* buf, int64_t cap) {
  if (!h || !buf || cap <= 0) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    const std::string s = h->eng->routes_json();
    if ((int64_t)s.size() + 1 > cap) return fail(ZASR_ERR_INVALID, "routes buffer too small");
    std::memcpy(buf, s.c_str(), s.size() + 1);
    return (int)ZASR_OK;
  });
}

int zasr_fbank_set_mel_banks(zasr_recognizer* h, const float* banks, int32_t n_bins) {
  if (!h || !banks) return fail(ZASR_ERR_INVALID, "null argument");
  if (n_bins != 256 && n_bins != 257) return fail(ZASR_ERR_INVALID, "n_bins must be 256 or 257");
  return guarded([&]() {
    std::lock_guard<std::mutex> lk(h->eng->mu);
    h->eng->set_mel_banks(banks, n_bins);
    return (int)ZASR_OK;
  });
}

int zasr_selftest_launch(int32_t block_threads) {
  if (block_threads <= 0) return fail(ZASR_ERR_INVALID, "block_threads must be positive");
  return guarded([&]() {
    zasr::launch_selftest_noop(block_threads);
    return (int)ZASR_OK;
  });
}

int zasr_selftest_gemm_h3r(int32_t M, int32_t K, int32_t N, int32_t epi, const float* A,
                           const float* W, const float* bias, float* C) {
  if (!A || !W || !C) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    zasr::selftest_gemm_h3r(M, K, N, epi, A, W, bias, C);
    return (int)ZASR_OK;
  });
}

int zasr_selftest_ffn_h3(int32_t R, int32_t D, int32_t F, const float* Y, const float* W1,
                         const float* b1, const float* W2, const float* b2,
                         const float* byp_orig, const float* byp_scale, float* X) {
  if (!Y || !W1 || !b1 || !W2 || !b2 || !X) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    zasr::selftest_ffn_h3(R, D, F, Y, W1, b1, W2, b2, byp_orig, byp_scale, X);
    return (int)ZASR_OK;
  });
}

int zasr_selftest_ffn_bf16(int32_t R, int32_t D, int32_t F, const float* W1, const float* b1,
                           const float* W2, const float* b2, const float* byp_orig,
                           const float* byp_scale, float* X, int32_t form) {
  if (!W1 || !b1 || !W2 || !b2 || !X) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    zasr::selftest_ffn_bf16(R, D, F, W1, b1, W2, b2, byp_orig, byp_scale, X, form);
    return (int)ZASR_OK;
  });
}

int zasr_silence_flags(const float* d_wav, int64_t n, int32_t frame_len, float threshold,
                       uint8_t* d_flags, void* stream) {
  if (n < 0 || (n > 0 && (!d_wav || !d_flags))) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    zasr::launch_silence_flags(d_wav, (long)n, (int)frame_len, threshold, d_flags,
                               reinterpret_cast<hipStream_t>(stream));
    return (int)ZASR_OK;
  });
}

// ---- offline streams (sherpa-onnx OfflineStream surface) ----
int zasr_set_tokens(zasr_recognizer* h, const char* tokens_path) {
  if (!h || !tokens_path) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    std::ifstream f(tokens_path);
    if (!f) return fail(ZASR_ERR_NOT_FOUND, std::string("tokens file not found: ") + tokens_path);
    std::lock_guard<std::mutex> lk(h->sym_mu);
    h->tokens_path = tokens_path;
    h->syms.reset();  // readers holding the old table keep it alive
    return (int)ZASR_OK;
  });
}

int zasr_create_stream(zasr_recognizer* h, zasr_stream** out) {
  if (!h || !out) return fail(ZASR_ERR_INVALID, "null argument");
  return guarded([&]() {
    auto* s = new zasr_stream;
    s->rec = h;
    *out = s;
    return (int)ZASR_OK;
  });
}

void zasr_destroy_stream(zasr_stream* s) { delete s; }

int zasr_stream_accept_waveform(zasr_stream* s, int32_t sample_rate, const float* samples,
                                int64_t n) {
  if (!s || n < 0 || (n > 0 && !samples)) return fail(ZASR_ERR_INVALID, "null argument");
  if (sample_rate != 16000) return fail(ZASR_ERR_INVALID, "sample rate must be 16000");
  if (s->decoded) return fail(ZASR_ERR_INVALID, "stream already decoded");
  return guarded([&]() {
    s->samples.insert(s->samples.end(), samples, samples + n);
    return (int)ZASR_OK;
  });
}

int zasr_decode_stream(zasr_recognizer* h, zasr_stream* s) {
  return zasr_decode_streams(h, &s, 1);
}

int zasr_decode_streams(zasr_recognizer* h, zasr_stream* const* ss, int32_t n) {
  if (!h || n < 0 || (n > 0 && !ss)) return fail(ZASR_ERR_INVALID, "null argument");
  for (int32_t i = 0; i < n; ++i) {
    if (!ss[i]) return fail(ZASR_ERR_INVALID, "null stream");
    if (ss[i]->rec != h) return fail(ZASR_ERR_INVALID, "stream belongs to another recognizer");
    for (int32_t j = 0; j < i; ++j)
      if (ss[j] == ss[i]) return fail(ZASR_ERR_INVALID, "stream listed twice");
  }
  return guarded([&]() {
    decode_streams_impl(h, ss, n);
    return (int)ZASR_OK;
  });
}

int32_t zasr_stream_is_decoded(const zasr_stream* s) { return s && s->decoded ? 1 : 0; }
int32_t zasr_stream_num_tokens(const zasr_stream* s) {
  return s ? (int32_t)s->res.tok.size() : 0;
}
int32_t zasr_stream_num_frames(const zasr_stream* s) { return s ? s->res.t_out : 0; }
const int32_t* zasr_stream_tokens(const zasr_stream* s) { return s ? s->res.tok.data() : nullptr; }
const int32_t* zasr_stream_frames(const zasr_stream* s) { return s ? s->res.frame.data() : nullptr; }
const double* zasr_stream_log_probs(const zasr_stream* s) { return s ? s->res.lp.data() : nullptr; }
const float* zasr_stream_token_stats(const zasr_stream* s) {
  return s ? s->res.stats.data() : nullptr;
}

int zasr_stream_result_json(const zasr_stream* s, char* buf, int64_t cap, int64_t* needed) {
  if (!s || !needed) return fail(ZASR_ERR_INVALID, "null argument");
  if (!s->decoded) return fail(ZASR_ERR_INVALID, "stream not decoded");
  return guarded([&]() {
    const std::shared_ptr<const std::vector<std::string>> tab = symbols(s->rec);
    const std::vector<std::string>& sym = *tab;
    const TokenResult& r = s->res;
    std::ostringstream os;
    std::string text;
    std::vector<std::string> toks;
    for (int t : r.tok) {
      toks.push_back(t >= 0 && t < (int)sym.size() ? sym[t] : std::string());
      text += toks.back();
    }
    os << "{\"lang\": \"\", \"emotion\": \"\", \"event\": \"\", \"text\": ";
    json_string(os, text);
    os << ", \"timestamps\": [";
    char b[40];
    for (size_t i = 0; i < r.frame.size(); ++i) {
      // frame shift 10 ms x subsampling 4 (sherpa-onnx OfflineRecognitionResult timestamps)
      std::snprintf(b, sizeof b, "%s%.2f", i ? ", " : "", (float)(0.04f * (float)r.frame[i]));
      os << b;
    }
    os << "], \"tokens\": [";
    for (size_t i = 0; i < toks.size(); ++i) {
      if (i) os << ", ";
      json_string(os, toks[i]);
    }
    os << "], \"ys_log_probs\": [";
    for (size_t i = 0; i < r.lp.size(); ++i) {
      std::snprintf(b, sizeof b, "%s%.17g", i ? ", " : "", r.lp[i]);
      os << b;
    }
    os << "], \"words\": []}";
    const std::string js = os.str();
    *needed = (int64_t)js.size() + 1;
    if (!buf || cap < *needed) return fail(ZASR_ERR_INVALID, "result buffer too small");
    std::memcpy(buf, js.c_str(), js.size() + 1);
    return (int)ZASR_OK;
  });
}

const char* zasr_last_error(void) { return g_last_error.c_str(); }
const char* zasr_version(void) { return "zasr 0.1 (gfx950)"; }

}  // extern "C"
