// ViBERT-capu punctuation / capitalization engine: the BERT encoder +
// Seq2Labels heads the reference runs with onnxruntime (core/gec_model.py:366-412; graph:
// convert_onnx/export_vibert_onnx.py Seq2LabelsModel) on MI355X -- exact-f32 MFMA GEMMs for
// the projections, LDS attention, LayerNorm kernels.  Host-side tokenization, the label
// vocabulary and the 3 refinement iterations stay the reference's Python.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace zasr {

class VibertEngine {
 public:
  VibertEngine(const std::string& model_dir, int device);
  ~VibertEngine();
  int num_labels() const { return labels_; }
  int num_detect() const { return detect_; }
  // the ONNX session's run(): int64 [B][L] inputs, [B][W] offsets -> logits [B][W][labels],
  // detect_logits [B][W][detect] (host buffers)
  void run_host(const long* input_ids, const long* attention_mask, const long* token_type_ids,
                const long* input_offsets, int B, int L, int W, float* logits, float* detect);
  std::mutex mu;

 private:
  struct Lin {
    float* w = nullptr;
    float* b = nullptr;
    int N = 0, K = 0;
  };
  struct Layer {
    Lin qkv, ao, inter, out;
    float *ln1_g, *ln1_b, *ln2_g, *ln2_b;
  };
  template <class T>
  T* ws(const std::string& name, size_t count);
  void gemm(const Lin& l, const float* A, int M, float* C, int epi);

  int device_ = 0, H_ = 0, heads_ = 0, inter_ = 0, labels_ = 0, detect_ = 0, max_pos_ = 0;
  long vocab_ = 0, type_vocab_ = 0;  // embedding rows (id range checks in run_host)
  float eps_ = 1e-12f;
  hipStream_t st_ = nullptr;
  float *word_ = nullptr, *pos_ = nullptr, *type_ = nullptr, *eln_g_ = nullptr, *eln_b_ = nullptr;
  std::vector<Layer> layers_;
  Lin heads_lin_;  // classifier rows then detector rows
  std::vector<void*> allocs_;
  std::map<std::string, std::pair<void*, size_t>> ws_;
};

}  // namespace zasr
