// Host-side weight containers for the ddmi runtime (see weights.cpp).
#pragma once
#include <initializer_list>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace ddmi {

constexpr size_t kNone = ~size_t(0);

struct HostTensor {
  std::vector<int64_t> shape;
  const float* data = nullptr;
  size_t numel = 0;
};

class BlobIndex {
 public:
  BlobIndex(const void* blob, size_t bytes);
  const HostTensor& get(const std::string& name, std::initializer_list<int64_t> shape) const;
  bool has(const std::string& name) const;

 private:
  std::unordered_map<std::string, HostTensor> map_;
};

// Host staging of all prepared weights, uploaded once into one device allocation.
class Arena {
 public:
  size_t add(const float* data, size_t n);
  size_t add(const std::vector<float>& v);
  size_t add_zero(size_t n);  // n zero floats, 64-byte aligned
  float* host(size_t off) { return host_.data() + off; }
  void upload();
  const float* ptr(size_t off) const { return off == kNone ? nullptr : dev_ + off; }
  size_t bytes() const { return host_.size() * sizeof(float); }
  ~Arena();

 private:
  std::vector<float> host_;
  float* dev_ = nullptr;
};

// f16x3 split copy of a [rows][K] fp32 B operand (conv_x3.hip): hi / lo fp16 images [rows][ldh]
// (ldh = K rounded up to 8, zero padded) stored in the float arena (2 halfs per slot), plus the
// per-row inverse power-of-two scale (float[rows]).
struct SplitW {
  size_t hi = kNone, lo = kNone, sinv = kNone;
  size_t b16 = kNone;  // bf16 image (RNE) of the same scaled weights, for DD_GEMM_BF16
  int ldh = 0;
};
// Conv weights re-laid out as [Cout][KH][KW][Cin_pad] (B operand "NK" of conv_gemm), BN folded.
struct Conv {
  size_t w = kNone, b = kNone;
  int cout = 0, cin = 0, cin_real = 0, k = 1, stride = 1, pad = 0;
  SplitW x3;
};
// nn.Linear weights [nout][nin].
struct Lin {
  size_t w = kNone, b = kNone;
  int nout = 0, nin = 0;
  SplitW x3;
};
struct LNp {
  size_t g = kNone, b = kNone;
  int c = 0;
};

Conv prep_conv(const BlobIndex& bx, Arena& ar, const std::string& wname, int cout, int cin, int k, int stride,
               int pad, const std::string& bn_prefix, const std::string& bias_name);
Lin prep_linear(const BlobIndex& bx, Arena& ar, const std::string& prefix, int nout, int nin, bool bias = true);
Lin prep_linear_rows(const BlobIndex& bx, Arena& ar, const std::string& wname, const std::string& bname,
                     int rows_total, int nin, int row0, int nrows);
// Split rows x K fp32 weights (host) into the f16x3 hi / lo images with per-row scale.
SplitW prep_split(Arena& ar, const float* w, int rows, int K);

LNp prep_ln(const BlobIndex& bx, Arena& ar, const std::string& prefix, int c);

}  // namespace ddmi
