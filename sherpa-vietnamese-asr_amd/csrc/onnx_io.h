// Reference model directories: the sherpa-onnx / icefall export the reference loads with
// onnxruntime (core/asr_engine.py:913-928: encoder-*.onnx, decoder-*.onnx, joiner-*.onnx,
// non-int8 preferred, an int8 file taken when it is the only one; tokens.txt beside them).
// This build does not run the ONNX graphs: it reads their initializers (a protobuf wire-format
// reader, no onnx / protobuf library), maps them onto the icefall state-dict names the engine
// uses (zasr/model.py::param_shapes), and infers the architecture from their shapes.
#pragma once
#include <string>
#include <vector>

#include "host_io.h"

namespace zasr {

// The three files create_recognizer would open (empty strings when one is missing).
struct OnnxFiles {
  std::string encoder, decoder, joiner;
  bool complete() const { return !encoder.empty() && !decoder.empty() && !joiner.empty(); }
};
OnnxFiles find_onnx_files(const std::string& model_dir);

// Loads the initializers of the three files into `out` under icefall names (f32; int8
// weights dequantized; MatMul operands stored transposed under torch.onnx's generated names
// are renamed from the bias of the Add that follows them and transposed back) and returns the
// model configuration as config.json text (ZipformerConfig fields), inferred from the shapes.
std::string load_onnx_model(const OnnxFiles& files, SafeTensors& out);

// The engine's weight set of a model directory: config.json + model.safetensors, or the
// reference's ONNX files.  Returns the config.json text.  Throws std::invalid_argument when
// neither form is present.
std::string load_model_dir(const std::string& dir, SafeTensors& out);

// The single-graph models of the other stages, kind "silero" | "campp" | "vibert":
// silero_vad_16k_op15.onnx (or silero_vad.onnx), campplus_cn_en_common_200k.onnx,
// vibert-capu.onnx (or vibert-capu.int8.onnx) -- the files the reference opens.  Returns the
// path in `dir` the reference would open, "" when none is there.
std::string find_stage_onnx(const std::string& dir, const std::string& kind);
// Loads one such file into the engine's tensor names (torch state-dict names) and returns the
// engine's <kind>_config.json text inferred from the graph (shapes, Conv attributes).
std::string load_stage_onnx(const std::string& path, const std::string& kind, SafeTensors& out);
// <kind>_config.json + the engine's safetensors file when present, else the reference .onnx.
// Throws std::invalid_argument when neither is in dir.
std::string load_stage_dir(const std::string& dir, const std::string& kind, SafeTensors& out);
// "silero_vad.safetensors" | "campp.safetensors" | "vibert.safetensors"
std::string stage_safetensors_name(const std::string& kind);

// Writes tensors as a float32 safetensors file (sorted names).
void write_safetensors(const std::string& path, const SafeTensors& t);

}  // namespace zasr
