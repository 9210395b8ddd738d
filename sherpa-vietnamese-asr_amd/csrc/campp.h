// CAM++ speaker-embedding engine: the reference runs the 3D-Speaker CAM++
// export through onnxruntime on batches of 1.5 s fbank windows
// (core/speaker_diarization_senko_campp_optimized.py:519-620, 86-159).  This is the same model
// (convert_onnx/export_campplus_onnx.py CAMPPlus, eval mode) on MI355X: FCM head as direct
// 2-D convolutions, the TDNN / dense-block projections on the exact-f32 MFMA GEMM, BatchNorm
// folded into the adjacent convolutions.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "gemm.h"
#include "kernels.h"

namespace zasr {

struct CamppConfig {
  int feat_dim = 80, emb = 192, growth = 32, bn_size = 4, init_ch = 128, m_ch = 32;
  std::vector<int> head_blocks{2, 2}, block_layers{12, 24, 16}, block_kernels{3, 3, 3},
      block_dil{1, 2, 2};
  int seg_len = 100;
};

class CamppEngine {
 public:
  CamppEngine(const std::string& model_dir, int device);
  ~CamppEngine();
  int emb_dim() const { return cfg_.emb; }

  // CAM++ fbank + per-utterance CMVN of one waveform (f32 in [-1, 1], 16 kHz):
  // [1 + (n - 400) / 160][80] (0 frames when n < 400)
  void fbank_host(const float* wav, long n, std::vector<float>& out);
  // embeddings of a (zero-padded) feature batch [N][T][80] -> [N][emb]
  void embed_host(const float* feats, int N, int T, float* out);
  void embed_device(const float* d_feats, int N, int T, float* d_out, hipStream_t st);
  // the front end of a whole file on the device (core/speaker_diarization_senko_campp_
  // optimized.py:540-600): fbank + per-region CMVN of every speech region [reg_off, +reg_len)
  // of d_wav in one launch, then the windows of `wf` frames every `sf` frames (tail pulled
  // back; a region shorter than a window is one window of all its frames, zero-padded to wf
  // like the reference's batch tensor; < 10 frames: none) gathered into d_feats [n][wf][80].
  // Returns n; win_* (host, capacity max_windows) get each window's region, first frame and
  // frame count.
  long windows_device(const float* d_wav, const long* reg_off, const long* reg_len, int nreg,
                      int wf, int sf, float* d_feats, long max_windows, int* win_region,
                      int* win_first, int* win_frames, hipStream_t st);

  std::mutex mu;

 private:
  struct Conv2 {
    float* w = nullptr;
    float* wk = nullptr;  // ci = 32: the MFMA kernel's weight image
    float *s = nullptr, *b = nullptr;
  };
  struct Lin {  // GEMM weight [N][K] (+ bias)
    float* w = nullptr;
    float* b = nullptr;
    int N = 0, K = 0;
  };
  struct DenseLayer {
    int cin = 0;
    float *bn1_s = nullptr, *bn1_b = nullptr;  // pre-activation of the block input
    Lin l1;                                     // 1 x 1, BN2 folded, ReLU epilogue
    Lin local;                                  // CAM linear_local, im2col order [o][k * bnc + c]
    float *m1w = nullptr, *m1b = nullptr, *m2w = nullptr, *m2b = nullptr;
  };
  struct Block {
    int cin0 = 0, cmax = 0, dil = 1, k = 3;
    std::vector<DenseLayer> layers;
    float *tr_s = nullptr, *tr_b = nullptr;
    Lin transit;
  };
  template <class T>
  T* ws(const std::string& name, size_t count);
  void gemm(const Lin& l, const float* A, int lda, int M, float* C, int ldc, int epi,
            const float* aux = nullptr, int ldaux = 0, int aload = 0,
            const float* a_scale = nullptr, const float* a_shift = nullptr,
            const GemmIm2col1d* i2c = nullptr);

  CamppConfig cfg_;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  hipStream_t st_ = nullptr;
  Conv2 c1_, c2_;
  struct ResBlock {
    Conv2 a, b, sc;
    bool has_sc = false;
    int stride = 1;
  };
  std::vector<ResBlock> res_;
  Lin tdnn_;
  std::vector<Block> blocks_;
  float *out_s_ = nullptr, *out_b_ = nullptr;
  Lin dense_;
  std::vector<void*> allocs_;
  std::map<std::string, std::pair<void*, size_t>> ws_;
  // fbank tables
  double* d_twiddle_ = nullptr;
  float* d_window_ = nullptr;
  int* d_mel_meta_ = nullptr;
  float* d_mel_w_ = nullptr;
};

}  // namespace zasr
