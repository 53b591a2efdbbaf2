// DDW1 weight-blob parser + host-side weight preparation (BatchNorm folding, OIHW -> OHWI
// re-layout with channel padding, in_proj slicing) for the ddmi runtime.
//
// The blob carries the reference V2TransfuserModel state dict (key schema of
// transfuser_model_v2.py / transfuser_backbone.py / timm resnet) as packed by
// diffusiondrive_amd/weights.py:pack_blob. Loading is strict: every key the hot path needs must
// be present with the expected shape (mirrors load_state_dict(strict=True),
// transfuser_agent.py:94-106).
#include "weights.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

namespace ddmi {

BlobIndex::BlobIndex(const void* blob, size_t bytes) {
  const uint8_t* p = static_cast<const uint8_t*>(blob);
  const uint8_t* end = p + bytes;
  auto need = [&](size_t n) {
    if (p > end || (size_t)(end - p) < n) throw std::invalid_argument("weight blob truncated");
  };
  // advance p to the next 16-byte boundary of the blob, never past its end
  auto align16 = [&]() {
    const size_t off = ((size_t)(p - static_cast<const uint8_t*>(blob)) + 15) & ~size_t(15);
    if (off > bytes) throw std::invalid_argument("weight blob truncated");
    p = static_cast<const uint8_t*>(blob) + off;
  };
  need(8);
  if (std::memcmp(p, "DDW1", 4) != 0) throw std::invalid_argument("weight blob: bad magic (expected DDW1)");
  uint32_t count;
  std::memcpy(&count, p + 4, 4);
  p += 8;
  for (uint32_t i = 0; i < count; ++i) {
    need(4);
    uint32_t nl;
    std::memcpy(&nl, p, 4);
    p += 4;
    need(nl);
    std::string name(reinterpret_cast<const char*>(p), nl);
    p += nl;
    need(4);
    uint32_t nd;
    std::memcpy(&nd, p, 4);
    p += 4;
    if (nd > 8) throw std::invalid_argument("weight blob: ndim > 8 for " + name);
    HostTensor t;
    need(8 * (size_t)nd);
    size_t numel = 1;
    for (uint32_t d = 0; d < nd; ++d) {
      int64_t v;
      std::memcpy(&v, p, 8);
      p += 8;
      if (v < 0) throw std::invalid_argument("weight blob: negative dim for " + name);
      if (v > 0 && numel > (SIZE_MAX / 4) / (size_t)v) throw std::invalid_argument("weight blob: tensor too large: " + name);
      t.shape.push_back(v);
      numel *= (size_t)v;
    }
    need(4);
    uint32_t dtype;
    std::memcpy(&dtype, p, 4);
    p += 4;
    if (dtype != 0) throw std::invalid_argument("weight blob: unsupported dtype for " + name);
    align16();
    need(numel * 4);
    t.data = reinterpret_cast<const float*>(p);
    t.numel = numel;
    p += numel * 4;
    align16();
    map_[name] = t;
  }
}

const HostTensor& BlobIndex::get(const std::string& name, std::initializer_list<int64_t> shape) const {
  auto it = map_.find(name);
  if (it == map_.end()) throw std::invalid_argument("missing weight: " + name);
  const HostTensor& t = it->second;
  std::vector<int64_t> want(shape);
  if (t.shape != want) {
    std::string s = "shape mismatch for " + name + ": got (";
    for (auto v : t.shape) s += std::to_string(v) + ",";
    s += ") expected (";
    for (auto v : want) s += std::to_string(v) + ",";
    throw std::invalid_argument(s + ")");
  }
  return t;
}

bool BlobIndex::has(const std::string& name) const { return map_.count(name) != 0; }

size_t Arena::add(const float* data, size_t n) {
  size_t off = host_.size();
  host_.insert(host_.end(), data, data + n);
  host_.resize((host_.size() + 15) & ~size_t(15), 0.f);  // 64-byte alignment for every tensor
  return off;
}

size_t Arena::add(const std::vector<float>& v) { return add(v.data(), v.size()); }

size_t Arena::add_zero(size_t n) {
  size_t off = host_.size();
  host_.resize(off + n, 0.f);
  host_.resize((host_.size() + 15) & ~size_t(15), 0.f);
  return off;
}

// f16x3 weight split (conv_x3.hip header): per row r, s_r = 2^e with max|w_r| * s_r in
// [2^14, 2^15] (exact power-of-two scaling, no fp16 overflow, lo parts clear of the subnormal
// range); hi = f16(w * s_r), lo = f16(w * s_r - hi), both RNE; sinv[r] = 1 / s_r.
SplitW prep_split(Arena& ar, const float* w, int rows, int K) {
  SplitW x;
  x.ldh = (K + 7) / 8 * 8;
  const size_t nh = (size_t)rows * x.ldh;  // halfs per image
  x.hi = ar.add_zero((nh + 1) / 2);
  x.lo = ar.add_zero((nh + 1) / 2);
  x.b16 = ar.add_zero((nh + 1) / 2);
  std::vector<float> sinv(rows, 1.f);
  _Float16* hi = reinterpret_cast<_Float16*>(ar.host(x.hi));
  _Float16* lo = reinterpret_cast<_Float16*>(ar.host(x.lo));
  __bf16* b16 = reinterpret_cast<__bf16*>(ar.host(x.b16));
  for (int r = 0; r < rows; ++r) {
    float amax = 0.f;
    for (int k = 0; k < K; ++k) amax = std::max(amax, std::fabs(w[(size_t)r * K + k]));
    int e = 0;
    if (amax > 0.f && std::isfinite(amax)) {
      int ex;
      std::frexp(amax, &ex);  // amax = f * 2^ex, f in [0.5, 1)
      e = 15 - ex;            // amax * 2^e in [2^14, 2^15)
    }
    const float s = std::ldexp(1.0f, e);
    sinv[r] = std::ldexp(1.0f, -e);
    for (int k = 0; k < K; ++k) {
      const float v = w[(size_t)r * K + k] * s;
      const _Float16 h = (_Float16)v;
      hi[(size_t)r * x.ldh + k] = h;
      lo[(size_t)r * x.ldh + k] = (_Float16)(v - (float)h);
      b16[(size_t)r * x.ldh + k] = (__bf16)v;
    }
  }
  x.sinv = ar.add(sinv);
  return x;
}

void Arena::upload() {
  if (dev_) DD_HIP_CHECK(hipFree(dev_));
  DD_HIP_CHECK(hipMalloc(&dev_, std::max<size_t>(host_.size(), 16) * sizeof(float)));
  DD_HIP_CHECK(hipMemcpy(dev_, host_.data(), host_.size() * sizeof(float), hipMemcpyHostToDevice));
}

Arena::~Arena() {
  if (dev_) (void)hipFree(dev_);
}

// conv weight OIHW (+ optional BN) -> [Cout][KH][KW][Cin_pad], folded bias.
Conv prep_conv(const BlobIndex& bx, Arena& ar, const std::string& wname, int cout, int cin, int k, int stride,
               int pad, const std::string& bn_prefix, const std::string& bias_name) {
  const HostTensor& w = bx.get(wname, {cout, cin, k, k});
  const int cin_p = (cin + 3) / 4 * 4;
  std::vector<double> scale(cout, 1.0), shift(cout, 0.0);
  if (!bn_prefix.empty()) {
    const HostTensor& g = bx.get(bn_prefix + ".weight", {cout});
    const HostTensor& b = bx.get(bn_prefix + ".bias", {cout});
    const HostTensor& m = bx.get(bn_prefix + ".running_mean", {cout});
    const HostTensor& v = bx.get(bn_prefix + ".running_var", {cout});
    for (int o = 0; o < cout; ++o) {
      const double s = (double)g.data[o] / std::sqrt((double)v.data[o] + 1e-5);
      scale[o] = s;
      shift[o] = (double)b.data[o] - (double)m.data[o] * s;
    }
  }
  if (!bias_name.empty()) {
    const HostTensor& b = bx.get(bias_name, {cout});
    for (int o = 0; o < cout; ++o) shift[o] += (double)b.data[o];
  }
  std::vector<float> wl((size_t)cout * k * k * cin_p, 0.f);
  for (int o = 0; o < cout; ++o)
    for (int i = 0; i < cin; ++i)
      for (int y = 0; y < k; ++y)
        for (int x = 0; x < k; ++x)
          wl[(((size_t)o * k + y) * k + x) * cin_p + i] =
              (float)((double)w.data[(((size_t)o * cin + i) * k + y) * k + x] * scale[o]);
  std::vector<float> bl(cout);
  bool any_bias = !bn_prefix.empty() || !bias_name.empty();
  for (int o = 0; o < cout; ++o) bl[o] = (float)shift[o];
  Conv c;
  c.x3 = prep_split(ar, wl.data(), cout, k * k * cin_p);
  c.w = ar.add(wl);
  c.b = any_bias ? ar.add(bl) : kNone;
  c.cout = cout;
  c.cin = cin_p;
  c.cin_real = cin;
  c.k = k;
  c.stride = stride;
  c.pad = pad;
  return c;
}

Lin prep_linear(const BlobIndex& bx, Arena& ar, const std::string& prefix, int nout, int nin, bool bias) {
  const HostTensor& w = bx.get(prefix + ".weight", {nout, nin});
  Lin l;
  l.w = ar.add(w.data, w.numel);
  l.x3 = prep_split(ar, w.data, nout, nin);
  l.b = bias ? ar.add(bx.get(prefix + ".bias", {nout}).data, (size_t)nout) : kNone;
  l.nout = nout;
  l.nin = nin;
  return l;
}

Lin prep_linear_rows(const BlobIndex& bx, Arena& ar, const std::string& wname, const std::string& bname, int rows_total,
                     int nin, int row0, int nrows) {
  const HostTensor& w = bx.get(wname, {rows_total, nin});
  const HostTensor& b = bx.get(bname, {rows_total});
  Lin l;
  l.w = ar.add(w.data + (size_t)row0 * nin, (size_t)nrows * nin);
  l.x3 = prep_split(ar, w.data + (size_t)row0 * nin, nrows, nin);
  l.b = ar.add(b.data + row0, (size_t)nrows);
  l.nout = nrows;
  l.nin = nin;
  return l;
}

LNp prep_ln(const BlobIndex& bx, Arena& ar, const std::string& prefix, int c) {
  LNp l;
  l.g = ar.add(bx.get(prefix + ".weight", {c}).data, (size_t)c);
  l.b = ar.add(bx.get(prefix + ".bias", {c}).data, (size_t)c);
  l.c = c;
  return l;
}

}  // namespace ddmi
