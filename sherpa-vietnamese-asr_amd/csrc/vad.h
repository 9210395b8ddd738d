// Silero VAD engine: the silero-vad v5 16 kHz network that the reference
// runs one 512-sample window per onnxruntime call (core/vad_utils.py:62-111), batched on
// MI355X.  Everything but the LSTM recurrence is computed for every window of every file at
// once (STFT and encoder convs as exact-f32 MFMA GEMMs, the LSTM input projection as one GEMM);
// the recurrence runs one workgroup per file.  Segmentation of the probabilities stays host
// logic (zasr/vad_utils.py).
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace zasr {

class VadEngine {
 public:
  VadEngine(const std::string& model_dir, int device);
  ~VadEngine();
  // speech probability of every full 512-sample window of every file (files concatenated in
  // d_audio at off[i], len[i] samples; probs of file i at d_probs[sum_{k<i} len[k] / 512]).
  // auto_boost: scale quiet files to a 0.071 peak first (core/vad_utils.py:203-208).
  // All pointers are device pointers except off / len.
  void probs_device(const float* d_audio, const long* off, const long* len, int n_files,
                    bool auto_boost, float* d_probs, hipStream_t user_stream);
  // the ORT session's single step for n independent streams: input [n][576], state [2][n][128]
  // -> prob [n], state_out [2][n][128] (host buffers)
  void window_host(const float* input, const float* state, int n, float* prob, float* state_out);
  // host-buffer variant of probs_device
  void probs_host(const float* audio, const long* off, const long* len, int n_files,
                  bool auto_boost, float* probs);
  // passes the last recurrence took (1 = every segment verified after the warm-up pass)
  int last_passes() const { return last_passes_; }
  std::mutex mu;

 private:
  struct Lin {
    float* w = nullptr;
    float* b = nullptr;
    int N = 0, K = 0;
  };
  template <class T>
  T* ws(const std::string& name, size_t count);
  void gemm(const Lin& l, const float* A, long M, float* C, int ldc, int epi);
  // encoder + LSTM input projection for n windows whose frames are in ws "frames" -> ws "gx"
  float* encode(long n);
  // the LSTM over files (first window, window count), parallel in time with exact verification
  void recurrence(const float* GX, const std::vector<long>& f_start, const std::vector<int>& f_count,
                  long nw, float* d_probs);

  int device_ = 0, bins_ = 129, kp1_ = 388, cus_ = 256, last_passes_ = 0;
  bool pit_ = true;  // ZASR_VAD_PIT=0: one sequential workgroup per file
  hipStream_t st_ = nullptr;
  Lin stft_;
  std::vector<Lin> conv_;
  std::vector<int> cin_, stride_;
  Lin ih_;
  float *whh_ = nullptr, *bhh_ = nullptr, *wd_ = nullptr;
  float bd_ = 0.f;
  std::vector<void*> allocs_;
  std::map<std::string, std::pair<void*, size_t>> ws_;
};

}  // namespace zasr
