#include "host_io.h"

#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <sys/stat.h>

namespace zasr {

namespace {

struct Parser {
  const std::string& s;
  size_t i = 0;
  explicit Parser(const std::string& t) : s(t) {}
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("json: ") + what + " at offset " + std::to_string(i));
  }
  Json value() {
    ws();
    if (i >= s.size()) fail("unexpected end");
    char c = s[i];
    Json j;
    if (c == '{') {
      j.kind = Json::OBJ;
      ++i;
      ws();
      if (i < s.size() && s[i] == '}') {
        ++i;
        return j;
      }
      for (;;) {
        ws();
        std::string k = string_lit();
        ws();
        if (i >= s.size() || s[i] != ':') fail("expected ':'");
        ++i;
        j.obj[k] = value();
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == '}') {
          ++i;
          break;
        }
        fail("expected ',' or '}'");
      }
    } else if (c == '[') {
      j.kind = Json::ARR;
      ++i;
      ws();
      if (i < s.size() && s[i] == ']') {
        ++i;
        return j;
      }
      for (;;) {
        j.arr.push_back(value());
        ws();
        if (i < s.size() && s[i] == ',') {
          ++i;
          continue;
        }
        if (i < s.size() && s[i] == ']') {
          ++i;
          break;
        }
        fail("expected ',' or ']'");
      }
    } else if (c == '"') {
      j.kind = Json::STR;
      j.str = string_lit();
    } else if (s.compare(i, 4, "true") == 0) {
      j.kind = Json::BOOL;
      j.b = true;
      i += 4;
    } else if (s.compare(i, 5, "false") == 0) {
      j.kind = Json::BOOL;
      i += 5;
    } else if (s.compare(i, 4, "null") == 0) {
      i += 4;
    } else {
      j.kind = Json::NUM;
      size_t st = i;
      while (i < s.size() && (std::isdigit((unsigned char)s[i]) || s[i] == '-' || s[i] == '+' ||
                              s[i] == '.' || s[i] == 'e' || s[i] == 'E'))
        ++i;
      if (st == i) fail("bad value");
      j.num = std::stod(s.substr(st, i - st));
    }
    return j;
  }
  std::string string_lit() {
    if (i >= s.size() || s[i] != '"') fail("expected string");
    ++i;
    std::string out;
    while (i < s.size() && s[i] != '"') {
      if (s[i] == '\\' && i + 1 < s.size()) {
        char e = s[i + 1];
        if (e == 'u') {  // keep escaped code units verbatim (names are ASCII here)
          out += s.substr(i, 6);
          i += 6;
          continue;
        }
        out += (e == 'n') ? '\n' : (e == 't') ? '\t' : e;
        i += 2;
        continue;
      }
      out += s[i++];
    }
    if (i >= s.size()) fail("unterminated string");
    ++i;
    return out;
  }
};

}  // namespace

Json Json::parse(const std::string& text) {
  Parser p(text);
  return p.value();
}

const Json& Json::at(const std::string& k) const {
  auto it = obj.find(k);
  if (kind != OBJ || it == obj.end()) throw std::runtime_error("json: missing key " + k);
  return it->second;
}

std::vector<int> Json::as_int_vec() const {
  std::vector<int> v;
  for (const auto& e : arr) v.push_back((int)e.num);
  return v;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

bool file_exists(const std::string& path) {
  struct stat st;
  return ::stat(path.c_str(), &st) == 0;
}

void SafeTensors::load(const std::string& path) {
  std::string raw = read_file(path);
  buf_.assign(raw.begin(), raw.end());
  if (buf_.size() < 8) throw std::runtime_error("safetensors: file too small");
  uint64_t hlen = 0;
  std::memcpy(&hlen, buf_.data(), 8);
  if (8 + hlen > buf_.size()) throw std::runtime_error("safetensors: bad header length");
  Json hdr = Json::parse(std::string(buf_.data() + 8, hlen));
  const char* data = buf_.data() + 8 + hlen;
  size_t data_len = buf_.size() - 8 - hlen;
  // convert non-f32 tensors into an owned f32 arena first (sizes known from the header)
  size_t extra = 0;
  for (const auto& kv : hdr.obj) {
    if (kv.first == "__metadata__") continue;
    const Json& t = kv.second;
    size_t n = 1;
    for (const auto& d : t.at("shape").arr) n *= (size_t)d.num;
    if (t.at("dtype").str != "F32") extra += n;
  }
  converted_.resize(extra);
  size_t conv_pos = 0;
  for (const auto& kv : hdr.obj) {
    if (kv.first == "__metadata__") continue;
    const Json& t = kv.second;
    HostTensor ht;
    for (const auto& d : t.at("shape").arr) ht.shape.push_back((int64_t)d.num);
    ht.numel = 1;
    for (auto d : ht.shape) ht.numel *= (size_t)d;
    size_t a = (size_t)t.at("data_offsets").arr[0].num;
    size_t b = (size_t)t.at("data_offsets").arr[1].num;
    if (b > data_len || a > b) throw std::runtime_error("safetensors: bad offsets for " + kv.first);
    const std::string& dt = t.at("dtype").str;
    if (dt == "F32") {
      if (b - a != ht.numel * 4) throw std::runtime_error("safetensors: size mismatch " + kv.first);
      ht.data = reinterpret_cast<const float*>(data + a);
    } else if (dt == "F64") {
      if (b - a != ht.numel * 8) throw std::runtime_error("safetensors: size mismatch " + kv.first);
      float* dst = converted_.data() + conv_pos;
      for (size_t k = 0; k < ht.numel; ++k) {
        double v;
        std::memcpy(&v, data + a + 8 * k, 8);
        dst[k] = (float)v;
      }
      ht.data = dst;
      conv_pos += ht.numel;
    } else {
      throw std::runtime_error("safetensors: unsupported dtype " + dt + " for " + kv.first);
    }
    tensors_[kv.first] = ht;
  }
}

void SafeTensors::put(const std::string& name, std::vector<int64_t> shape, std::vector<float>&& data) {
  size_t n = 1;
  for (auto d : shape) n *= (size_t)d;
  if (n != data.size()) throw std::runtime_error("tensor " + name + ": shape / data size mismatch");
  owned_.push_back(std::move(data));
  HostTensor ht;
  ht.shape = std::move(shape);
  ht.numel = n;
  ht.data = owned_.back().data();
  tensors_[name] = ht;
}

const HostTensor& SafeTensors::get(const std::string& name) const {
  auto it = tensors_.find(name);
  if (it == tensors_.end()) throw std::runtime_error("model: missing tensor " + name);
  return it->second;
}

}  // namespace zasr
