// Host-side file formats: a small JSON reader (config.json, safetensors headers) and a
// safetensors loader.  No third-party dependencies.
#pragma once
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace zasr {

struct Json {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  double num = 0.0;
  std::string str;
  std::vector<Json> arr;
  std::map<std::string, Json> obj;

  static Json parse(const std::string& text);
  const Json& at(const std::string& k) const;
  bool has(const std::string& k) const { return kind == OBJ && obj.count(k) != 0; }
  long as_int() const { return (long)num; }
  std::vector<int> as_int_vec() const;
};

struct HostTensor {
  std::vector<int64_t> shape;
  const float* data = nullptr;
  size_t numel = 0;
};

// A named f32 tensor set: a safetensors file (load) and/or tensors added by put (owned).
class SafeTensors {
 public:
  void load(const std::string& path);
  void put(const std::string& name, std::vector<int64_t> shape, std::vector<float>&& data);
  bool has(const std::string& name) const { return tensors_.count(name) != 0; }
  const HostTensor& get(const std::string& name) const;
  const std::map<std::string, HostTensor>& all() const { return tensors_; }

 private:
  std::vector<char> buf_;
  std::vector<float> converted_;
  std::deque<std::vector<float>> owned_;
  std::map<std::string, HostTensor> tensors_;
};

std::string read_file(const std::string& path);
bool file_exists(const std::string& path);

}  // namespace zasr
