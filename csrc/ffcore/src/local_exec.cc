#include "ff/local_exec.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <functional>
#include <numeric>
#include <random>

namespace ff {

void HostTensor::resize(const std::vector<int64_t>& d) {
  dims = d;
  int64_t n = 1;
  for (auto x : d) n *= x;
  v.assign(static_cast<size_t>(n), 0.f);
}

namespace {

using Ctx = LocalTrainingBacking::OpCtx;

int64_t last_dim(const HostTensor& t) { return t.dims.empty() ? 1 : t.dims.back(); }

float act_f(Activation a, float x) {
  switch (a) {
    case Activation::RELU: return x > 0.f ? x : 0.f;
    case Activation::SIGMOID: return 1.f / (1.f + std::exp(-x));
    case Activation::TANH: return std::tanh(x);
    case Activation::GELU: {
      const float k = 0.7978845608028654f;
      return 0.5f * x * (1.f + std::tanh(k * (x + 0.044715f * x * x * x)));
    }
    default: return x;
  }
}
// derivative w.r.t. the pre-activation x
float act_d(Activation a, float x) {
  switch (a) {
    case Activation::RELU: return x > 0.f ? 1.f : 0.f;
    case Activation::SIGMOID: {
      const float s = 1.f / (1.f + std::exp(-x));
      return s * (1.f - s);
    }
    case Activation::TANH: {
      const float t = std::tanh(x);
      return 1.f - t * t;
    }
    case Activation::GELU: {
      const float k = 0.7978845608028654f;
      const float u = k * (x + 0.044715f * x * x * x);
      const float t = std::tanh(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
    }
    default: return 1.f;
  }
}

Activation op_act(OpType t) {
  switch (t) {
    case OpType::RELU: return Activation::RELU;
    case OpType::SIGMOID: return Activation::SIGMOID;
    case OpType::TANH: return Activation::TANH;
    case OpType::GELU: return Activation::GELU;
    default: return Activation::NONE;
  }
}

// C[M,N] (+)= A[M,K] * B[K,N] with optional transposes (row-major)
void matmul(const float* A, const float* B, float* C, int64_t M, int64_t N, int64_t K, bool ta, bool tb,
            bool accumulate) {
  if (!accumulate) std::fill(C, C + M * N, 0.f);
  for (int64_t i = 0; i < M; ++i) {
    float* c = C + i * N;
    for (int64_t k = 0; k < K; ++k) {
      const float a = ta ? A[k * M + i] : A[i * K + k];
      if (a == 0.f) continue;
      if (!tb) {
        const float* b = B + k * N;
        for (int64_t j = 0; j < N; ++j) c[j] += a * b[j];
      } else {
        for (int64_t j = 0; j < N; ++j) c[j] += a * B[j * K + k];
      }
    }
  }
}

void add_into(HostTensor* d, const std::vector<float>& g) {
  if (!d) return;
  for (size_t i = 0; i < g.size(); ++i) d->v[i] += g[i];
}

// ---- LINEAR: y = act(x W + b), W [in, out]
void linear_fwd(Ctx& c) {
  const HostTensor& x = *c.in[0];
  const HostTensor& W = *c.w[0];
  HostTensor& y = *c.out[0];
  const int64_t in = W.dims[0], out = W.dims[1], rows = x.numel() / in;
  matmul(x.v.data(), W.v.data(), y.v.data(), rows, out, in, false, false, false);
  if (c.w.size() > 1)
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t j = 0; j < out; ++j) y.v[r * out + j] += c.w[1]->v[j];
  const Activation a = activation_from_string(c.op->s("activation"));
  if (a != Activation::NONE) {
    c.saved->assign(1, y);  // pre-activation
    for (auto& e : y.v) e = act_f(a, e);
  }
}
void linear_bwd(Ctx& c) {
  const HostTensor& x = *c.in[0];
  const HostTensor& W = *c.w[0];
  const int64_t in = W.dims[0], out = W.dims[1], rows = x.numel() / in;
  std::vector<float> g = c.d_out[0]->v;
  const Activation a = activation_from_string(c.op->s("activation"));
  if (a != Activation::NONE) {
    const auto& pre = (*c.saved)[0].v;
    for (size_t i = 0; i < g.size(); ++i) g[i] *= act_d(a, pre[i]);
  }
  if (c.d_w[0]) matmul(x.v.data(), g.data(), c.d_w[0]->v.data(), in, out, rows, true, false, true);
  if (c.w.size() > 1 && c.d_w[1])
    for (int64_t r = 0; r < rows; ++r)
      for (int64_t j = 0; j < out; ++j) c.d_w[1]->v[j] += g[r * out + j];
  if (c.d_in[0]) matmul(g.data(), W.v.data(), c.d_in[0]->v.data(), rows, in, out, false, true, true);
}

// ---- element-wise activations
void act_fwd(Ctx& c) {
  const Activation a = op_act(c.op->type);
  auto& y = c.out[0]->v;
  const auto& x = c.in[0]->v;
  for (size_t i = 0; i < x.size(); ++i) y[i] = act_f(a, x[i]);
}
void act_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const Activation a = op_act(c.op->type);
  const auto& x = c.in[0]->v;
  const auto& g = c.d_out[0]->v;
  for (size_t i = 0; i < x.size(); ++i) c.d_in[0]->v[i] += g[i] * act_d(a, x[i]);
}

// ---- binary element-wise (equal shapes)
void binary_fwd(Ctx& c) {
  const auto& a = c.in[0]->v;
  const auto& b = c.in[1]->v;
  if (a.size() != b.size()) throw FFError("local execution: broadcasting binaries are not supported");
  auto& y = c.out[0]->v;
  for (size_t i = 0; i < a.size(); ++i) {
    switch (c.op->type) {
      case OpType::EW_ADD: y[i] = a[i] + b[i]; break;
      case OpType::EW_SUB: y[i] = a[i] - b[i]; break;
      case OpType::EW_MUL: y[i] = a[i] * b[i]; break;
      case OpType::EW_DIV: y[i] = a[i] / b[i]; break;
      case OpType::EW_MAX: y[i] = std::max(a[i], b[i]); break;
      case OpType::EW_MIN: y[i] = std::min(a[i], b[i]); break;
      default: throw FFError("local execution: bad binary op");
    }
  }
}
void binary_bwd(Ctx& c) {
  const auto& a = c.in[0]->v;
  const auto& b = c.in[1]->v;
  const auto& g = c.d_out[0]->v;
  for (size_t i = 0; i < a.size(); ++i) {
    float ga = 0.f, gb = 0.f;
    switch (c.op->type) {
      case OpType::EW_ADD: ga = g[i]; gb = g[i]; break;
      case OpType::EW_SUB: ga = g[i]; gb = -g[i]; break;
      case OpType::EW_MUL: ga = g[i] * b[i]; gb = g[i] * a[i]; break;
      case OpType::EW_DIV: ga = g[i] / b[i]; gb = -g[i] * a[i] / (b[i] * b[i]); break;
      case OpType::EW_MAX: (a[i] >= b[i] ? ga : gb) = g[i]; break;
      case OpType::EW_MIN: (a[i] <= b[i] ? ga : gb) = g[i]; break;
      default: break;
    }
    if (c.d_in[0]) c.d_in[0]->v[i] += ga;
    if (c.d_in[1]) c.d_in[1]->v[i] += gb;
  }
}

// ---- scalar ops
void scalar_fwd(Ctx& c) {
  const float s = static_cast<float>(c.op->f("scalar"));
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  for (size_t i = 0; i < x.size(); ++i) {
    switch (c.op->type) {
      case OpType::SCALAR_MULTIPLY: y[i] = x[i] * s; break;
      case OpType::SCALAR_ADD: y[i] = x[i] + s; break;
      case OpType::SCALAR_SUB: y[i] = x[i] - s; break;
      case OpType::SCALAR_TRUE_DIV: y[i] = x[i] / s; break;
      default: y[i] = x[i];
    }
  }
}
void scalar_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  float k = 1.f;
  if (c.op->type == OpType::SCALAR_MULTIPLY) k = static_cast<float>(c.op->f("scalar"));
  if (c.op->type == OpType::SCALAR_TRUE_DIV) k = 1.f / static_cast<float>(c.op->f("scalar"));
  const auto& g = c.d_out[0]->v;
  for (size_t i = 0; i < g.size(); ++i) c.d_in[0]->v[i] += k * g[i];
}

// ---- copies (flat / reshape / identity / dropout in inference)
void copy_fwd(Ctx& c) { c.out[0]->v = c.in[0]->v; }
void copy_bwd(Ctx& c) { add_into(c.d_in[0], c.d_out[0]->v); }

// ---- dropout: counter-hash mask, scaled by 1/(1-p)
float hash_uniform(uint64_t seed, uint64_t i) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);
}
void dropout_fwd(Ctx& c) {
  const float p = static_cast<float>(c.op->f("rate"));
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  if (!c.training || p <= 0.f) {
    y = x;
    return;
  }
  for (size_t i = 0; i < x.size(); ++i) y[i] = hash_uniform(c.seed, i) < p ? 0.f : x[i] / (1.f - p);
}
void dropout_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const float p = static_cast<float>(c.op->f("rate"));
  const auto& g = c.d_out[0]->v;
  for (size_t i = 0; i < g.size(); ++i)
    c.d_in[0]->v[i] += (p > 0.f && hash_uniform(c.seed, i) < p) ? 0.f : g[i] / (1.f - p);
}

// ---- softmax over the last dim
void softmax_fwd(Ctx& c) {
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  const int64_t C = last_dim(*c.in[0]), R = static_cast<int64_t>(x.size()) / C;
  for (int64_t r = 0; r < R; ++r) {
    const float* xr = x.data() + r * C;
    float* yr = y.data() + r * C;
    const float m = *std::max_element(xr, xr + C);
    double s = 0;
    for (int64_t j = 0; j < C; ++j) s += (yr[j] = std::exp(xr[j] - m));
    for (int64_t j = 0; j < C; ++j) yr[j] = static_cast<float>(yr[j] / s);
  }
}
void softmax_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const auto& y = c.out[0]->v;
  const auto& g = c.d_out[0]->v;
  const int64_t C = last_dim(*c.out[0]), R = static_cast<int64_t>(y.size()) / C;
  for (int64_t r = 0; r < R; ++r) {
    double dot = 0;
    for (int64_t j = 0; j < C; ++j) dot += g[r * C + j] * y[r * C + j];
    for (int64_t j = 0; j < C; ++j) c.d_in[0]->v[r * C + j] += y[r * C + j] * (g[r * C + j] - static_cast<float>(dot));
  }
}

// ---- layer norm over trailing axes (affine gamma/beta)
void layernorm_fwd(Ctx& c) {
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  const auto axes = c.op->ints("axes");
  int64_t N = 1;
  const int nd = static_cast<int>(c.in[0]->dims.size());
  for (auto a : axes) N *= c.in[0]->dims[(a % nd + nd) % nd];
  const int64_t R = static_cast<int64_t>(x.size()) / N;
  const float eps = static_cast<float>(c.op->f("eps"));
  c.saved->assign(2, HostTensor{});
  (*c.saved)[0].v.resize(R);  // mean
  (*c.saved)[1].v.resize(R);  // rstd
  for (int64_t r = 0; r < R; ++r) {
    double s = 0, s2 = 0;
    for (int64_t j = 0; j < N; ++j) s += x[r * N + j];
    const double mean = s / N;
    for (int64_t j = 0; j < N; ++j) {
      const double d = x[r * N + j] - mean;
      s2 += d * d;
    }
    const float rstd = static_cast<float>(1.0 / std::sqrt(s2 / N + eps));
    (*c.saved)[0].v[r] = static_cast<float>(mean);
    (*c.saved)[1].v[r] = rstd;
    for (int64_t j = 0; j < N; ++j) {
      float v = (x[r * N + j] - static_cast<float>(mean)) * rstd;
      if (!c.w.empty()) v = v * c.w[0]->v[j] + (c.w.size() > 1 ? c.w[1]->v[j] : 0.f);
      y[r * N + j] = v;
    }
  }
}
void layernorm_bwd(Ctx& c) {
  const auto& x = c.in[0]->v;
  const auto& g = c.d_out[0]->v;
  const auto& mean = (*c.saved)[0].v;
  const auto& rstd = (*c.saved)[1].v;
  const int64_t R = static_cast<int64_t>(mean.size()), N = static_cast<int64_t>(x.size()) / R;
  for (int64_t r = 0; r < R; ++r) {
    double s1 = 0, s2 = 0;
    for (int64_t j = 0; j < N; ++j) {
      const float xh = (x[r * N + j] - mean[r]) * rstd[r];
      const float gg = g[r * N + j] * (c.w.empty() ? 1.f : c.w[0]->v[j]);
      s1 += gg;
      s2 += gg * xh;
      if (!c.w.empty() && c.d_w[0]) c.d_w[0]->v[j] += g[r * N + j] * xh;
      if (c.w.size() > 1 && c.d_w[1]) c.d_w[1]->v[j] += g[r * N + j];
    }
    if (!c.d_in[0]) continue;
    for (int64_t j = 0; j < N; ++j) {
      const float xh = (x[r * N + j] - mean[r]) * rstd[r];
      const float gg = g[r * N + j] * (c.w.empty() ? 1.f : c.w[0]->v[j]);
      c.d_in[0]->v[r * N + j] += rstd[r] * (gg - static_cast<float>(s1 / N) - xh * static_cast<float>(s2 / N));
    }
  }
}

// ---- embedding (aggr none / sum / avg); indices carried as floats
void embedding_fwd(Ctx& c) {
  const auto& idx = c.in[0]->v;
  const HostTensor& W = *c.w[0];
  const int64_t D = W.dims[1], E = W.dims[0];
  const std::string aggr = c.op->s("aggr");
  auto& y = c.out[0]->v;
  std::fill(y.begin(), y.end(), 0.f);
  const int64_t L = aggr == "none" ? 1 : last_dim(*c.in[0]);
  const int64_t B = static_cast<int64_t>(idx.size()) / L;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t l = 0; l < L; ++l) {
      const int64_t e = static_cast<int64_t>(idx[b * L + l]);
      if (e < 0 || e >= E) throw FFError("local execution: embedding index out of range");
      const float s = aggr == "avg" ? 1.f / static_cast<float>(L) : 1.f;
      for (int64_t d = 0; d < D; ++d) y[b * D + d] += s * W.v[e * D + d];
    }
}
void embedding_bwd(Ctx& c) {
  if (!c.d_w[0]) return;
  const auto& idx = c.in[0]->v;
  const int64_t D = c.w[0]->dims[1];
  const std::string aggr = c.op->s("aggr");
  const int64_t L = aggr == "none" ? 1 : last_dim(*c.in[0]);
  const int64_t B = static_cast<int64_t>(idx.size()) / L;
  const auto& g = c.d_out[0]->v;
  for (int64_t b = 0; b < B; ++b)
    for (int64_t l = 0; l < L; ++l) {
      const int64_t e = static_cast<int64_t>(idx[b * L + l]);
      const float s = aggr == "avg" ? 1.f / static_cast<float>(L) : 1.f;
      for (int64_t d = 0; d < D; ++d) c.d_w[0]->v[e * D + d] += s * g[b * D + d];
    }
}

// ---- concat / split along an axis: [outer, len_i, inner] blocks
void concat_fwd(Ctx& c) {
  const int nd = static_cast<int>(c.out[0]->dims.size());
  const int ax = static_cast<int>((c.op->i("axis") % nd + nd) % nd);
  int64_t outer = 1, inner = 1;
  for (int d = 0; d < ax; ++d) outer *= c.out[0]->dims[d];
  for (int d = ax + 1; d < nd; ++d) inner *= c.out[0]->dims[d];
  const int64_t tot = c.out[0]->dims[ax];
  int64_t off = 0;
  for (auto* in : c.in) {
    const int64_t len = in->dims[ax];
    for (int64_t o = 0; o < outer; ++o)
      std::copy(in->v.begin() + o * len * inner, in->v.begin() + (o + 1) * len * inner,
                c.out[0]->v.begin() + (o * tot + off) * inner);
    off += len;
  }
}
void concat_bwd(Ctx& c) {
  const int nd = static_cast<int>(c.out[0]->dims.size());
  const int ax = static_cast<int>((c.op->i("axis") % nd + nd) % nd);
  int64_t outer = 1, inner = 1;
  for (int d = 0; d < ax; ++d) outer *= c.out[0]->dims[d];
  for (int d = ax + 1; d < nd; ++d) inner *= c.out[0]->dims[d];
  const int64_t tot = c.out[0]->dims[ax];
  int64_t off = 0;
  for (size_t i = 0; i < c.in.size(); ++i) {
    const int64_t len = c.in[i]->dims[ax];
    if (c.d_in[i])
      for (int64_t o = 0; o < outer; ++o)
        for (int64_t k = 0; k < len * inner; ++k) c.d_in[i]->v[o * len * inner + k] += c.d_out[0]->v[(o * tot + off) * inner + k];
    off += len;
  }
}

// ---- batch matmul [.., M, K] x [.., K, N]
void bmm_fwd(Ctx& c) {
  const HostTensor& a = *c.in[0];
  const HostTensor& b = *c.in[1];
  const int nd = static_cast<int>(a.dims.size());
  const int64_t M = a.dims[nd - 2], K = a.dims[nd - 1], N = b.dims[nd - 1];
  const int64_t B = a.numel() / (M * K);
  for (int64_t i = 0; i < B; ++i)
    matmul(a.v.data() + i * M * K, b.v.data() + i * K * N, c.out[0]->v.data() + i * M * N, M, N, K, false, false,
           false);
}
void bmm_bwd(Ctx& c) {
  const HostTensor& a = *c.in[0];
  const HostTensor& b = *c.in[1];
  const int nd = static_cast<int>(a.dims.size());
  const int64_t M = a.dims[nd - 2], K = a.dims[nd - 1], N = b.dims[nd - 1];
  const int64_t B = a.numel() / (M * K);
  const float* g = c.d_out[0]->v.data();
  for (int64_t i = 0; i < B; ++i) {
    if (c.d_in[0]) matmul(g + i * M * N, b.v.data() + i * K * N, c.d_in[0]->v.data() + i * M * K, M, K, N, false, true, true);
    if (c.d_in[1]) matmul(a.v.data() + i * M * K, g + i * M * N, c.d_in[1]->v.data() + i * K * N, K, N, M, true, false, true);
  }
}

// ---- math unaries (exp, sin, cos, rsqrt, sqrt, log, pow, elu)
float math_f(const OpAttrs& op, float x) {
  switch (op.type) {
    case OpType::EXP: return std::exp(x);
    case OpType::SIN: return std::sin(x);
    case OpType::COS: return std::cos(x);
    case OpType::RSQRT: return 1.f / std::sqrt(x);
    case OpType::SQRT: return std::sqrt(x);
    case OpType::LOG: return std::log(x);
    case OpType::POW: return std::pow(x, static_cast<float>(op.f("exponent")));
    case OpType::ELU: return x > 0.f ? x : std::exp(x) - 1.f;
    default: return x;
  }
}
float math_d(const OpAttrs& op, float x) {
  switch (op.type) {
    case OpType::EXP: return std::exp(x);
    case OpType::SIN: return std::cos(x);
    case OpType::COS: return -std::sin(x);
    case OpType::RSQRT: return -0.5f / (x * std::sqrt(x));
    case OpType::SQRT: return 0.5f / std::sqrt(x);
    case OpType::LOG: return 1.f / x;
    case OpType::POW: {
      const float e = static_cast<float>(op.f("exponent"));
      return e * std::pow(x, e - 1.f);
    }
    case OpType::ELU: return x > 0.f ? 1.f : std::exp(x);
    default: return 1.f;
  }
}
void math_fwd(Ctx& c) {
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  for (size_t i = 0; i < x.size(); ++i) y[i] = math_f(*c.op, x[i]);
}
void math_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const auto& x = c.in[0]->v;
  const auto& g = c.d_out[0]->v;
  for (size_t i = 0; i < x.size(); ++i) c.d_in[0]->v[i] += g[i] * math_d(*c.op, x[i]);
}

std::vector<int64_t> strides_of(const std::vector<int64_t>& d) {
  std::vector<int64_t> s(d.size(), 1);
  for (int i = static_cast<int>(d.size()) - 2; i >= 0; --i) s[i] = s[i + 1] * d[i + 1];
  return s;
}
int norm_dim(int64_t d, size_t nd) { return static_cast<int>(d < 0 ? d + static_cast<int64_t>(nd) : d); }

// ---- transpose: y[i_0..] = x[perm-indexed]
void transpose_map(const Ctx& c, const std::function<void(int64_t, int64_t)>& f) {
  const auto& xd = c.in[0]->dims;
  const auto& p = c.op->ints("perm");
  const auto xs = strides_of(xd);
  const auto& yd = c.out[0]->dims;
  const int nd = static_cast<int>(yd.size());
  std::vector<int64_t> idx(nd, 0);
  const int64_t n = c.out[0]->numel();
  for (int64_t o = 0; o < n; ++o) {
    int64_t src = 0;
    for (int k = 0; k < nd; ++k) src += idx[k] * xs[norm_dim(p[k], xd.size())];
    f(o, src);
    for (int k = nd - 1; k >= 0; --k) {
      if (++idx[k] < yd[k]) break;
      idx[k] = 0;
    }
  }
}
void transpose_fwd(Ctx& c) { transpose_map(c, [&](int64_t o, int64_t s) { c.out[0]->v[o] = c.in[0]->v[s]; }); }
void transpose_bwd(Ctx& c) {
  if (c.d_in[0]) transpose_map(c, [&](int64_t o, int64_t s) { c.d_in[0]->v[s] += c.d_out[0]->v[o]; });
}

// ---- reverse along one axis (an involution: the backward is the same map)
void reverse_map(const Ctx& c, const std::function<void(int64_t, int64_t)>& f) {
  const auto& d = c.in[0]->dims;
  const int ax = norm_dim(c.op->i("axis"), d.size());
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < ax; ++k) outer *= d[k];
  for (size_t k = ax + 1; k < d.size(); ++k) inner *= d[k];
  const int64_t L = d[ax];
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t l = 0; l < L; ++l)
      for (int64_t i = 0; i < inner; ++i) f((o * L + l) * inner + i, (o * L + (L - 1 - l)) * inner + i);
}
void reverse_fwd(Ctx& c) { reverse_map(c, [&](int64_t o, int64_t s) { c.out[0]->v[o] = c.in[0]->v[s]; }); }
void reverse_bwd(Ctx& c) {
  if (c.d_in[0]) reverse_map(c, [&](int64_t o, int64_t s) { c.d_in[0]->v[s] += c.d_out[0]->v[o]; });
}

// ---- split along an axis
void split_fwd(Ctx& c) {
  const auto& d = c.in[0]->dims;
  const int ax = norm_dim(c.op->i("axis"), d.size());
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < ax; ++k) outer *= d[k];
  for (size_t k = ax + 1; k < d.size(); ++k) inner *= d[k];
  int64_t off = 0;
  for (size_t j = 0; j < c.out.size(); ++j) {
    const int64_t L = c.out[j]->dims[ax];
    for (int64_t o = 0; o < outer; ++o)
      std::copy_n(c.in[0]->v.begin() + (o * d[ax] + off) * inner, L * inner, c.out[j]->v.begin() + o * L * inner);
    off += L;
  }
}
void split_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const auto& d = c.in[0]->dims;
  const int ax = norm_dim(c.op->i("axis"), d.size());
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < ax; ++k) outer *= d[k];
  for (size_t k = ax + 1; k < d.size(); ++k) inner *= d[k];
  int64_t off = 0;
  for (size_t j = 0; j < c.out.size(); ++j) {
    const int64_t L = c.out[j]->dims[ax];
    if (c.d_out[j])
      for (int64_t o = 0; o < outer; ++o)
        for (int64_t e = 0; e < L * inner; ++e)
          c.d_in[0]->v[(o * d[ax] + off) * inner + e] += c.d_out[j]->v[o * L * inner + e];
    off += L;
  }
}

// ---- reduce sum / mean over axes
void reduce_map(const Ctx& c, const std::function<void(int64_t, int64_t)>& f) {
  const auto& d = c.in[0]->dims;
  std::vector<bool> red(d.size(), false);
  for (auto a : c.op->ints("axes")) red[norm_dim(a, d.size())] = true;
  std::vector<int64_t> od;
  for (size_t k = 0; k < d.size(); ++k) od.push_back(red[k] ? 1 : d[k]);
  const auto os = strides_of(od);
  std::vector<int64_t> idx(d.size(), 0);
  const int64_t n = c.in[0]->numel();
  for (int64_t i = 0; i < n; ++i) {
    int64_t o = 0;
    for (size_t k = 0; k < d.size(); ++k) o += (red[k] ? 0 : idx[k]) * os[k];
    f(i, o);
    for (int k = static_cast<int>(d.size()) - 1; k >= 0; --k) {
      if (++idx[k] < d[k]) break;
      idx[k] = 0;
    }
  }
}
double reduce_scale(const Ctx& c) {
  if (c.op->type != OpType::MEAN && c.op->type != OpType::REDUCE_MEAN) return 1.0;
  return static_cast<double>(c.out[0]->numel()) / static_cast<double>(std::max<int64_t>(1, c.in[0]->numel()));
}
void reduce_fwd(Ctx& c) {
  std::fill(c.out[0]->v.begin(), c.out[0]->v.end(), 0.f);
  reduce_map(c, [&](int64_t i, int64_t o) { c.out[0]->v[o] += c.in[0]->v[i]; });
  const float k = static_cast<float>(reduce_scale(c));
  if (k != 1.f)
    for (auto& e : c.out[0]->v) e *= k;
}
void reduce_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const float k = static_cast<float>(reduce_scale(c));
  reduce_map(c, [&](int64_t i, int64_t o) { c.d_in[0]->v[i] += k * c.d_out[0]->v[o]; });
}

// ---- gather along `dim` (index has the input's rank)
void gather_map(const Ctx& c, const std::function<void(int64_t, int64_t)>& f) {
  const auto& xd = c.in[0]->dims;
  const auto& id = c.in[1]->dims;
  const int dim = norm_dim(c.op->i("dim"), xd.size());
  const auto xs = strides_of(xd);
  std::vector<int64_t> idx(id.size(), 0);
  const int64_t n = c.in[1]->numel();
  for (int64_t o = 0; o < n; ++o) {
    int64_t src = 0;
    for (size_t k = 0; k < id.size(); ++k) {
      int64_t v = static_cast<int>(k) == dim ? static_cast<int64_t>(c.in[1]->v[o]) : idx[k];
      v = std::min<int64_t>(std::max<int64_t>(v, 0), xd[k] - 1);
      src += v * xs[k];
    }
    f(o, src);
    for (int k = static_cast<int>(id.size()) - 1; k >= 0; --k) {
      if (++idx[k] < id[k]) break;
      idx[k] = 0;
    }
  }
}
void gather_fwd(Ctx& c) { gather_map(c, [&](int64_t o, int64_t s) { c.out[0]->v[o] = c.in[0]->v[s]; }); }
void gather_bwd(Ctx& c) {
  if (c.d_in[0]) gather_map(c, [&](int64_t o, int64_t s) { c.d_in[0]->v[s] += c.d_out[0]->v[o]; });
}

// ---- conv2d, NCHW, weight [O, C/g, KH, KW] (direct convolution)
struct ConvGeom {
  int64_t N, C, H, W, O, OH, OW, KH, KW, SH, SW, PH, PW, G;
};
ConvGeom conv_geom(const Ctx& c) {
  const auto& x = c.in[0]->dims;
  const auto& y = c.out[0]->dims;
  return {x[0], x[1], x[2], x[3], y[1], y[2], y[3], c.op->i("kernel_h"), c.op->i("kernel_w"), c.op->i("stride_h"),
          c.op->i("stride_w"), c.op->i("padding_h"), c.op->i("padding_w"), c.op->i("groups")};
}
template <typename F>
void conv_loop(const ConvGeom& g, F&& f) {
  const int64_t cpg = g.C / g.G, opg = g.O / g.G;
  for (int64_t n = 0; n < g.N; ++n)
    for (int64_t o = 0; o < g.O; ++o) {
      const int64_t grp = o / opg;
      for (int64_t oh = 0; oh < g.OH; ++oh)
        for (int64_t ow = 0; ow < g.OW; ++ow) {
          const int64_t yi = ((n * g.O + o) * g.OH + oh) * g.OW + ow;
          for (int64_t ci = 0; ci < cpg; ++ci)
            for (int64_t kh = 0; kh < g.KH; ++kh) {
              const int64_t ih = oh * g.SH - g.PH + kh;
              if (ih < 0 || ih >= g.H) continue;
              for (int64_t kw = 0; kw < g.KW; ++kw) {
                const int64_t iw = ow * g.SW - g.PW + kw;
                if (iw < 0 || iw >= g.W) continue;
                const int64_t xi = ((n * g.C + grp * cpg + ci) * g.H + ih) * g.W + iw;
                const int64_t wi = ((o * cpg + ci) * g.KH + kh) * g.KW + kw;
                f(yi, xi, wi);
              }
            }
        }
    }
}
void conv2d_fwd(Ctx& c) {
  const auto g = conv_geom(c);
  auto& y = c.out[0]->v;
  std::fill(y.begin(), y.end(), 0.f);
  const auto& x = c.in[0]->v;
  const auto& w = c.w[0]->v;
  conv_loop(g, [&](int64_t yi, int64_t xi, int64_t wi) { y[yi] += x[xi] * w[wi]; });
  if (c.w.size() > 1)
    for (int64_t i = 0; i < static_cast<int64_t>(y.size()); ++i) y[i] += c.w[1]->v[(i / (g.OH * g.OW)) % g.O];
  const Activation a = activation_from_string(c.op->s("activation"));
  if (a != Activation::NONE) {
    c.saved->assign(1, *c.out[0]);
    for (auto& e : y) e = act_f(a, e);
  }
}
void conv2d_bwd(Ctx& c) {
  const auto g = conv_geom(c);
  std::vector<float> gy = c.d_out[0]->v;
  const Activation a = activation_from_string(c.op->s("activation"));
  if (a != Activation::NONE)
    for (size_t i = 0; i < gy.size(); ++i) gy[i] *= act_d(a, (*c.saved)[0].v[i]);
  const auto& x = c.in[0]->v;
  const auto& w = c.w[0]->v;
  conv_loop(g, [&](int64_t yi, int64_t xi, int64_t wi) {
    if (c.d_w[0]) c.d_w[0]->v[wi] += gy[yi] * x[xi];
    if (c.d_in[0]) c.d_in[0]->v[xi] += gy[yi] * w[wi];
  });
  if (c.w.size() > 1 && c.d_w[1])
    for (int64_t i = 0; i < static_cast<int64_t>(gy.size()); ++i) c.d_w[1]->v[(i / (g.OH * g.OW)) % g.O] += gy[i];
}

// ---- pool2d (max / avg, padding excluded from the average)
void pool2d_fwd(Ctx& c) {
  const auto& xd = c.in[0]->dims;
  const auto& yd = c.out[0]->dims;
  const int64_t KH = c.op->i("kernel_h"), KW = c.op->i("kernel_w"), SH = c.op->i("stride_h"),
                SW = c.op->i("stride_w"), PH = c.op->i("padding_h"), PW = c.op->i("padding_w");
  const bool mx = c.op->s("pool_type") == "max";
  HostTensor arg;
  arg.resize(yd);
  for (int64_t nc = 0; nc < yd[0] * yd[1]; ++nc)
    for (int64_t oh = 0; oh < yd[2]; ++oh)
      for (int64_t ow = 0; ow < yd[3]; ++ow) {
        float acc = mx ? -INFINITY : 0.f;
        int64_t best = -1, cnt = 0;
        for (int64_t kh = 0; kh < KH; ++kh)
          for (int64_t kw = 0; kw < KW; ++kw) {
            const int64_t ih = oh * SH - PH + kh, iw = ow * SW - PW + kw;
            if (ih < 0 || ih >= xd[2] || iw < 0 || iw >= xd[3]) continue;
            const int64_t xi = (nc * xd[2] + ih) * xd[3] + iw;
            const float v = c.in[0]->v[xi];
            if (mx) {
              if (v > acc) acc = v, best = xi;
            } else {
              acc += v;
              ++cnt;
            }
          }
        const int64_t yi = (nc * yd[2] + oh) * yd[3] + ow;
        c.out[0]->v[yi] = mx ? acc : acc / static_cast<float>(std::max<int64_t>(1, cnt));
        arg.v[yi] = static_cast<float>(mx ? best : cnt);
      }
  c.saved->assign(1, arg);
  const Activation a = activation_from_string(c.op->s("activation"));
  if (a != Activation::NONE) {
    c.saved->push_back(*c.out[0]);
    for (auto& e : c.out[0]->v) e = act_f(a, e);
  }
}
void pool2d_bwd(Ctx& c) {
  if (!c.d_in[0]) return;
  const auto& xd = c.in[0]->dims;
  const auto& yd = c.out[0]->dims;
  const int64_t KH = c.op->i("kernel_h"), KW = c.op->i("kernel_w"), SH = c.op->i("stride_h"),
                SW = c.op->i("stride_w"), PH = c.op->i("padding_h"), PW = c.op->i("padding_w");
  const bool mx = c.op->s("pool_type") == "max";
  const auto& arg = (*c.saved)[0].v;
  const Activation a = activation_from_string(c.op->s("activation"));
  for (int64_t nc = 0; nc < yd[0] * yd[1]; ++nc)
    for (int64_t oh = 0; oh < yd[2]; ++oh)
      for (int64_t ow = 0; ow < yd[3]; ++ow) {
        const int64_t yi = (nc * yd[2] + oh) * yd[3] + ow;
        float g = c.d_out[0]->v[yi];
        if (a != Activation::NONE) g *= act_d(a, (*c.saved)[1].v[yi]);
        if (mx) {
          if (arg[yi] >= 0) c.d_in[0]->v[static_cast<int64_t>(arg[yi])] += g;
          continue;
        }
        const float share = g / std::max(1.f, arg[yi]);
        for (int64_t kh = 0; kh < KH; ++kh)
          for (int64_t kw = 0; kw < KW; ++kw) {
            const int64_t ih = oh * SH - PH + kh, iw = ow * SW - PW + kw;
            if (ih < 0 || ih >= xd[2] || iw < 0 || iw >= xd[3]) continue;
            c.d_in[0]->v[(nc * xd[2] + ih) * xd[3] + iw] += share;
          }
      }
}

// ---- batch norm (training statistics over N and the spatial dims, channel dim 1)
void bn_geom(const Ctx& c, int64_t& N, int64_t& C, int64_t& S) {
  const auto& d = c.in[0]->dims;
  N = d[0];
  C = d[1];
  S = 1;
  for (size_t k = 2; k < d.size(); ++k) S *= d[k];
}
void batchnorm_fwd(Ctx& c) {
  int64_t N, C, S;
  bn_geom(c, N, C, S);
  const float eps = static_cast<float>(c.op->f("eps"));
  HostTensor stat;
  stat.resize({2, C});  // mean, inverse std
  const auto& x = c.in[0]->v;
  auto& y = c.out[0]->v;
  const double cnt = static_cast<double>(N * S);
  for (int64_t ch = 0; ch < C; ++ch) {
    double m = 0, v = 0;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t s = 0; s < S; ++s) m += x[(n * C + ch) * S + s];
    m /= cnt;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t s = 0; s < S; ++s) {
        const double dd = x[(n * C + ch) * S + s] - m;
        v += dd * dd;
      }
    v /= cnt;
    const float inv = 1.f / std::sqrt(static_cast<float>(v) + eps);
    stat.v[ch] = static_cast<float>(m);
    stat.v[C + ch] = inv;
    const float gm = c.w.empty() ? 1.f : c.w[0]->v[ch], bt = c.w.size() > 1 ? c.w[1]->v[ch] : 0.f;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t s = 0; s < S; ++s) {
        const int64_t i = (n * C + ch) * S + s;
        float o = (x[i] - stat.v[ch]) * inv * gm + bt;
        if (c.op->b("relu") && o < 0.f) o = 0.f;
        y[i] = o;
      }
  }
  c.saved->assign(1, stat);
}
void batchnorm_bwd(Ctx& c) {
  int64_t N, C, S;
  bn_geom(c, N, C, S);
  const auto& x = c.in[0]->v;
  const auto& y = c.out[0]->v;
  const auto& st = (*c.saved)[0].v;
  const double cnt = static_cast<double>(N * S);
  for (int64_t ch = 0; ch < C; ++ch) {
    const float m = st[ch], inv = st[C + ch];
    const float gm = c.w.empty() ? 1.f : c.w[0]->v[ch];
    double sg = 0, sgx = 0;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t s = 0; s < S; ++s) {
        const int64_t i = (n * C + ch) * S + s;
        float g = c.d_out[0]->v[i];
        if (c.op->b("relu") && y[i] <= 0.f) g = 0.f;
        const float xh = (x[i] - m) * inv;
        sg += g;
        sgx += g * xh;
      }
    if (c.d_w.size() > 0 && c.d_w[0]) c.d_w[0]->v[ch] += static_cast<float>(sgx);
    if (c.d_w.size() > 1 && c.d_w[1]) c.d_w[1]->v[ch] += static_cast<float>(sg);
    if (!c.d_in[0]) continue;
    for (int64_t n = 0; n < N; ++n)
      for (int64_t s = 0; s < S; ++s) {
        const int64_t i = (n * C + ch) * S + s;
        float g = c.d_out[0]->v[i];
        if (c.op->b("relu") && y[i] <= 0.f) g = 0.f;
        const float xh = (x[i] - m) * inv;
        c.d_in[0]->v[i] += static_cast<float>(gm * inv * (g - sg / cnt - xh * sgx / cnt));
      }
  }
}

// ---- multi-head attention with the logical weight layout of op_attrs mha_spec:
// weight [P, H], per head column: Wq [Eq, k] | Wk [Ek, k] | Wv [Ev, v] | Wo [v, E]
// (row-major blocks); input bias [2k + v, H] (q | k | v); output bias [E].
struct MhaGeom {
  int64_t B, Sq, Sk, Eq, Ek, Ev, E, H, kd, vd;
  int64_t off_q() const { return 0; }
  int64_t off_k() const { return Eq * kd; }
  int64_t off_v() const { return Eq * kd + Ek * kd; }
  int64_t off_o() const { return Eq * kd + Ek * kd + Ev * vd; }
};
MhaGeom mha_geom(const Ctx& c) {
  MhaGeom g;
  g.B = c.in[0]->dims[0];
  g.Sq = c.in[0]->dims[1];
  g.Sk = c.in[1]->dims[1];
  g.Eq = c.in[0]->dims[2];
  g.Ek = c.in[1]->dims[2];
  g.Ev = c.in[2]->dims[2];
  g.E = c.op->i("embed_dim");
  g.H = c.op->i("num_heads");
  g.kd = c.op->i("kdim") > 0 ? c.op->i("kdim") : g.E / g.H;
  g.vd = c.op->i("vdim") > 0 ? c.op->i("vdim") : g.E / g.H;
  return g;
}
// dense [rows, cols] block of head h out of the [P, H] weight (or its gradient)
std::vector<float> head_block(const HostTensor& W, int64_t H, int64_t h, int64_t off, int64_t rows, int64_t cols) {
  std::vector<float> m(rows * cols);
  for (int64_t i = 0; i < rows * cols; ++i) m[i] = W.v[(off + i) * H + h];
  return m;
}
void head_block_add(HostTensor* W, int64_t H, int64_t h, int64_t off, const std::vector<float>& m) {
  if (!W) return;
  for (size_t i = 0; i < m.size(); ++i) W->v[(off + static_cast<int64_t>(i)) * H + h] += m[i];
}
void mha_fwd(Ctx& c) {
  const auto g = mha_geom(c);
  const bool bias = c.w.size() > 1, causal = c.op->b("causal");
  const float scale = 1.f / std::sqrt(static_cast<float>(g.kd));
  auto& y = c.out[0]->v;
  std::fill(y.begin(), y.end(), 0.f);
  c.saved->assign(5, HostTensor{});
  auto& Qs = (*c.saved)[0].v;
  auto& Ks = (*c.saved)[1].v;
  auto& Vs = (*c.saved)[2].v;
  auto& Ps = (*c.saved)[3].v;
  auto& Os = (*c.saved)[4].v;
  Qs.assign(g.B * g.H * g.Sq * g.kd, 0.f);
  Ks.assign(g.B * g.H * g.Sk * g.kd, 0.f);
  Vs.assign(g.B * g.H * g.Sk * g.vd, 0.f);
  Ps.assign(g.B * g.H * g.Sq * g.Sk, 0.f);
  Os.assign(g.B * g.H * g.Sq * g.vd, 0.f);
  for (int64_t h = 0; h < g.H; ++h) {
    const auto Wq = head_block(*c.w[0], g.H, h, g.off_q(), g.Eq, g.kd);
    const auto Wk = head_block(*c.w[0], g.H, h, g.off_k(), g.Ek, g.kd);
    const auto Wv = head_block(*c.w[0], g.H, h, g.off_v(), g.Ev, g.vd);
    const auto Wo = head_block(*c.w[0], g.H, h, g.off_o(), g.vd, g.E);
    for (int64_t b = 0; b < g.B; ++b) {
      const int64_t bh = b * g.H + h;
      float* Q = Qs.data() + bh * g.Sq * g.kd;
      float* K = Ks.data() + bh * g.Sk * g.kd;
      float* V = Vs.data() + bh * g.Sk * g.vd;
      float* P = Ps.data() + bh * g.Sq * g.Sk;
      float* O = Os.data() + bh * g.Sq * g.vd;
      matmul(c.in[0]->v.data() + b * g.Sq * g.Eq, Wq.data(), Q, g.Sq, g.kd, g.Eq, false, false, false);
      matmul(c.in[1]->v.data() + b * g.Sk * g.Ek, Wk.data(), K, g.Sk, g.kd, g.Ek, false, false, false);
      matmul(c.in[2]->v.data() + b * g.Sk * g.Ev, Wv.data(), V, g.Sk, g.vd, g.Ev, false, false, false);
      if (bias) {
        const auto& bi = c.w[1]->v;  // [2k + v, H]
        for (int64_t s = 0; s < g.Sq; ++s)
          for (int64_t j = 0; j < g.kd; ++j) Q[s * g.kd + j] += bi[j * g.H + h];
        for (int64_t s = 0; s < g.Sk; ++s) {
          for (int64_t j = 0; j < g.kd; ++j) K[s * g.kd + j] += bi[(g.kd + j) * g.H + h];
          for (int64_t j = 0; j < g.vd; ++j) V[s * g.vd + j] += bi[(2 * g.kd + j) * g.H + h];
        }
      }
      matmul(Q, K, P, g.Sq, g.Sk, g.kd, false, true, false);
      for (int64_t i = 0; i < g.Sq; ++i) {
        float* r = P + i * g.Sk;
        float m = -INFINITY;
        for (int64_t j = 0; j < g.Sk; ++j) {
          r[j] = (causal && j > i) ? -INFINITY : r[j] * scale;
          m = std::max(m, r[j]);
        }
        double sum = 0;
        for (int64_t j = 0; j < g.Sk; ++j) sum += (r[j] = r[j] == -INFINITY ? 0.f : std::exp(r[j] - m));
        for (int64_t j = 0; j < g.Sk; ++j) r[j] = static_cast<float>(r[j] / sum);
      }
      matmul(P, V, O, g.Sq, g.vd, g.Sk, false, false, false);
      matmul(O, Wo.data(), y.data() + b * g.Sq * g.E, g.Sq, g.E, g.vd, false, false, true);
    }
  }
  if (c.w.size() > 2)
    for (int64_t r = 0; r < g.B * g.Sq; ++r)
      for (int64_t e = 0; e < g.E; ++e) y[r * g.E + e] += c.w[2]->v[e];
}
void mha_bwd(Ctx& c) {
  const auto g = mha_geom(c);
  const bool bias = c.w.size() > 1;
  const float scale = 1.f / std::sqrt(static_cast<float>(g.kd));
  const auto& gy = c.d_out[0]->v;
  const auto& Qs = (*c.saved)[0].v;
  const auto& Ks = (*c.saved)[1].v;
  const auto& Vs = (*c.saved)[2].v;
  const auto& Ps = (*c.saved)[3].v;
  const auto& Os = (*c.saved)[4].v;
  HostTensor* dW = c.d_w[0];
  HostTensor* dbi = bias && c.d_w.size() > 1 ? c.d_w[1] : nullptr;
  if (c.w.size() > 2 && c.d_w.size() > 2 && c.d_w[2])
    for (int64_t r = 0; r < g.B * g.Sq; ++r)
      for (int64_t e = 0; e < g.E; ++e) c.d_w[2]->v[e] += gy[r * g.E + e];
  std::vector<float> dO(g.Sq * g.vd), dP(g.Sq * g.Sk), dQ(g.Sq * g.kd), dK(g.Sk * g.kd), dV(g.Sk * g.vd);
  for (int64_t h = 0; h < g.H; ++h) {
    const auto Wq = head_block(*c.w[0], g.H, h, g.off_q(), g.Eq, g.kd);
    const auto Wk = head_block(*c.w[0], g.H, h, g.off_k(), g.Ek, g.kd);
    const auto Wv = head_block(*c.w[0], g.H, h, g.off_v(), g.Ev, g.vd);
    const auto Wo = head_block(*c.w[0], g.H, h, g.off_o(), g.vd, g.E);
    std::vector<float> dWq(Wq.size(), 0.f), dWk(Wk.size(), 0.f), dWv(Wv.size(), 0.f), dWo(Wo.size(), 0.f);
    for (int64_t b = 0; b < g.B; ++b) {
      const int64_t bh = b * g.H + h;
      const float* Q = Qs.data() + bh * g.Sq * g.kd;
      const float* K = Ks.data() + bh * g.Sk * g.kd;
      const float* V = Vs.data() + bh * g.Sk * g.vd;
      const float* P = Ps.data() + bh * g.Sq * g.Sk;
      const float* O = Os.data() + bh * g.Sq * g.vd;
      const float* G = gy.data() + b * g.Sq * g.E;
      matmul(O, G, dWo.data(), g.vd, g.E, g.Sq, true, false, true);
      matmul(G, Wo.data(), dO.data(), g.Sq, g.vd, g.E, false, true, false);
      matmul(dO.data(), V, dP.data(), g.Sq, g.Sk, g.vd, false, true, false);
      matmul(P, dO.data(), dV.data(), g.Sk, g.vd, g.Sq, true, false, false);
      for (int64_t i = 0; i < g.Sq; ++i) {  // softmax backward, then the 1/sqrt(k) scale
        double dot = 0;
        for (int64_t j = 0; j < g.Sk; ++j) dot += P[i * g.Sk + j] * dP[i * g.Sk + j];
        for (int64_t j = 0; j < g.Sk; ++j)
          dP[i * g.Sk + j] = P[i * g.Sk + j] * (dP[i * g.Sk + j] - static_cast<float>(dot)) * scale;
      }
      matmul(dP.data(), K, dQ.data(), g.Sq, g.kd, g.Sk, false, false, false);
      matmul(dP.data(), Q, dK.data(), g.Sk, g.kd, g.Sq, true, false, false);
      const float* xq = c.in[0]->v.data() + b * g.Sq * g.Eq;
      const float* xk = c.in[1]->v.data() + b * g.Sk * g.Ek;
      const float* xv = c.in[2]->v.data() + b * g.Sk * g.Ev;
      matmul(xq, dQ.data(), dWq.data(), g.Eq, g.kd, g.Sq, true, false, true);
      matmul(xk, dK.data(), dWk.data(), g.Ek, g.kd, g.Sk, true, false, true);
      matmul(xv, dV.data(), dWv.data(), g.Ev, g.vd, g.Sk, true, false, true);
      if (c.d_in[0]) matmul(dQ.data(), Wq.data(), c.d_in[0]->v.data() + b * g.Sq * g.Eq, g.Sq, g.Eq, g.kd, false, true, true);
      if (c.d_in[1]) matmul(dK.data(), Wk.data(), c.d_in[1]->v.data() + b * g.Sk * g.Ek, g.Sk, g.Ek, g.kd, false, true, true);
      if (c.d_in[2]) matmul(dV.data(), Wv.data(), c.d_in[2]->v.data() + b * g.Sk * g.Ev, g.Sk, g.Ev, g.vd, false, true, true);
      if (dbi) {
        for (int64_t s = 0; s < g.Sq; ++s)
          for (int64_t j = 0; j < g.kd; ++j) dbi->v[j * g.H + h] += dQ[s * g.kd + j];
        for (int64_t s = 0; s < g.Sk; ++s) {
          for (int64_t j = 0; j < g.kd; ++j) dbi->v[(g.kd + j) * g.H + h] += dK[s * g.kd + j];
          for (int64_t j = 0; j < g.vd; ++j) dbi->v[(2 * g.kd + j) * g.H + h] += dV[s * g.vd + j];
        }
      }
    }
    head_block_add(dW, g.H, h, g.off_q(), dWq);
    head_block_add(dW, g.H, h, g.off_k(), dWk);
    head_block_add(dW, g.H, h, g.off_v(), dWv);
    head_block_add(dW, g.H, h, g.off_o(), dWo);
  }
}

double elapsed_ms(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

const std::map<OpType, LocalTrainingBacking::OpImpl>& LocalTrainingBacking::registry() {
  static const std::map<OpType, OpImpl> r = [] {
    std::map<OpType, OpImpl> m;
    m[OpType::LINEAR] = {linear_fwd, linear_bwd};
    for (auto t : {OpType::RELU, OpType::SIGMOID, OpType::TANH, OpType::GELU}) m[t] = {act_fwd, act_bwd};
    for (auto t : {OpType::EW_ADD, OpType::EW_SUB, OpType::EW_MUL, OpType::EW_DIV, OpType::EW_MAX, OpType::EW_MIN})
      m[t] = {binary_fwd, binary_bwd};
    for (auto t : {OpType::SCALAR_MULTIPLY, OpType::SCALAR_ADD, OpType::SCALAR_SUB, OpType::SCALAR_TRUE_DIV})
      m[t] = {scalar_fwd, scalar_bwd};
    for (auto t : {OpType::FLAT, OpType::RESHAPE, OpType::IDENTITY, OpType::NOOP}) m[t] = {copy_fwd, copy_bwd};
    m[OpType::DROPOUT] = {dropout_fwd, dropout_bwd};
    m[OpType::SOFTMAX] = {softmax_fwd, softmax_bwd};
    m[OpType::LAYERNORM] = {layernorm_fwd, layernorm_bwd};
    m[OpType::EMBEDDING] = {embedding_fwd, embedding_bwd};
    m[OpType::CONCAT] = {concat_fwd, concat_bwd};
    m[OpType::BATCHMATMUL] = {bmm_fwd, bmm_bwd};
    for (auto t : {OpType::EXP, OpType::SIN, OpType::COS, OpType::RSQRT, OpType::SQRT, OpType::LOG, OpType::POW,
                   OpType::ELU})
      m[t] = {math_fwd, math_bwd};
    m[OpType::TRANSPOSE] = {transpose_fwd, transpose_bwd};
    m[OpType::REVERSE] = {reverse_fwd, reverse_bwd};
    m[OpType::SPLIT] = {split_fwd, split_bwd};
    for (auto t : {OpType::REDUCE_SUM, OpType::REDUCE_MEAN, OpType::MEAN}) m[t] = {reduce_fwd, reduce_bwd};
    m[OpType::GATHER] = {gather_fwd, gather_bwd};
    m[OpType::CONV2D] = {conv2d_fwd, conv2d_bwd};
    m[OpType::POOL2D] = {pool2d_fwd, pool2d_bwd};
    m[OpType::BATCHNORM] = {batchnorm_fwd, batchnorm_bwd};
    m[OpType::MULTIHEAD_ATTENTION] = {mha_fwd, mha_bwd};
    return m;
  }();
  return r;
}

// ---------------------------------------------------------------------------
LocalTrainingBacking::LocalTrainingBacking(const ComputationGraph& cg, LocalOptimizer opt, std::string loss,
                                           uint64_t seed, bool input_grads)
    : cg_(cg), opt_(std::move(opt)), loss_(std::move(loss)), seed_(seed) {
  const auto& reg = registry();
  for (int n : cg_.layers_in_topo_order()) {
    const auto& node = cg_.g.node(n);
    const OpType t = node.label.op.type;
    for (size_t i = 0; i < node.outputs.size(); ++i) {
      ValueRef v{n, static_cast<int>(i)};
      val_[v].resize(node.outputs[i].shape.dims);
    }
    if (t == OpType::INPUT) {
      input_of_[node.label.name] = n;
      // fed tensors get no gradient (the reference's create_gradients=NO
      // marking of input-fed tensors) unless asked for (cost estimation)
      needs_grad_[{n, 0}] = input_grads && node.outputs[0].create_grad;
      continue;
    }
    if (t == OpType::WEIGHT) {
      weight_of_[node.label.name] = n;
      needs_grad_[{n, 0}] = node.outputs[0].create_grad;
      init_weight(n, val_[{n, 0}], node.outputs[0].initializer, seed_);
      continue;
    }
    if (!reg.count(t)) throw FFError("local execution: no CPU implementation for " + to_string(t));
    bool ng = false;
    for (auto const& v : node.inputs) ng = ng || needs_grad_[v];
    for (size_t i = 0; i < node.outputs.size(); ++i) needs_grad_[{n, static_cast<int>(i)}] = ng;
    order_.push_back(n);
  }
  if (order_.empty()) throw FFError("local execution: graph has no operators");
  output_ = {order_.back(), 0};
  const OpType last = cg_.g.node(order_.back()).label.op.type;
  fused_softmax_ce_ = last == OpType::SOFTMAX &&
                      (loss_ == "sparse_categorical_crossentropy" || loss_ == "categorical_crossentropy");
  for (auto const& kv : needs_grad_)
    if (kv.second) grad_[kv.first].resize(val_[kv.first].dims);
}

void LocalTrainingBacking::init_weight(int node, HostTensor& t, const std::string& init_json, uint64_t seed) {
  Json j = init_json.empty() ? Json::parse(R"({"type":"glorot_uniform"})") : Json::parse(init_json);
  const std::string type = j.contains("type") ? j["type"].as_string() : "glorot_uniform";
  std::mt19937_64 rng(seed * 1000003ull + static_cast<uint64_t>(node) +
                      (j.contains("seed") ? static_cast<uint64_t>(j["seed"].as_int()) : 0));
  const int64_t n = t.numel();
  if (type == "zero") {
    std::fill(t.v.begin(), t.v.end(), 0.f);
  } else if (type == "constant") {
    std::fill(t.v.begin(), t.v.end(), static_cast<float>(j.contains("value") ? j["value"].as_double() : 0.0));
  } else if (type == "uniform") {
    std::uniform_real_distribution<float> d(static_cast<float>(j["min"].as_double()),
                                            static_cast<float>(j["max"].as_double()));
    for (int64_t i = 0; i < n; ++i) t.v[i] = d(rng);
  } else if (type == "normal" || type == "truncated_normal") {
    const float mean = static_cast<float>(j.contains("mean") ? j["mean"].as_double() : 0.0);
    const float sd = static_cast<float>(j.contains("stddev") ? j["stddev"].as_double() : 1.0);
    std::normal_distribution<float> d(mean, sd);
    for (int64_t i = 0; i < n; ++i) {
      float x = d(rng);
      if (type == "truncated_normal")
        while (std::fabs(x - mean) > 2 * sd) x = d(rng);
      t.v[i] = x;
    }
  } else {  // glorot_uniform: fan_in = dims[0] (x receptive field), fan_out = dims[1]
    double fan_in = t.dims.size() > 0 ? static_cast<double>(t.dims[0]) : 1.0;
    double fan_out = t.dims.size() > 1 ? static_cast<double>(t.dims[1]) : fan_in;
    double rf = 1.0;
    for (size_t d = 2; d < t.dims.size(); ++d) rf *= static_cast<double>(t.dims[d]);
    const float lim = static_cast<float>(std::sqrt(6.0 / ((fan_in + fan_out) * rf)));
    std::uniform_real_distribution<float> d(-lim, lim);
    for (int64_t i = 0; i < n; ++i) t.v[i] = d(rng);
  }
}

std::vector<std::string> LocalTrainingBacking::input_names() const {
  std::vector<std::string> r;
  for (auto const& kv : input_of_) r.push_back(kv.first);
  return r;
}
std::vector<std::string> LocalTrainingBacking::weight_names() const {
  std::vector<std::string> r;
  for (auto const& kv : weight_of_) r.push_back(kv.first);
  return r;
}
std::vector<int64_t> LocalTrainingBacking::shape_of(const std::string& name) const {
  auto it = input_of_.find(name);
  if (it != input_of_.end()) return val_.at({it->second, 0}).dims;
  it = weight_of_.find(name);
  if (it != weight_of_.end()) return val_.at({it->second, 0}).dims;
  auto l = cg_.find_layer(name);
  if (!l) throw FFError("local execution: no tensor named " + name);
  return val_.at({*l, 0}).dims;
}
void LocalTrainingBacking::set_input(const std::string& name, const std::vector<float>& data) {
  auto it = input_of_.find(name);
  if (it == input_of_.end()) throw FFError("local execution: no input named " + name);
  auto& t = val_[{it->second, 0}];
  if (static_cast<int64_t>(data.size()) != t.numel()) throw FFError("local execution: input " + name + " size mismatch");
  t.v = data;
}
void LocalTrainingBacking::set_weight(const std::string& name, const std::vector<float>& data) {
  auto it = weight_of_.find(name);
  if (it == weight_of_.end()) throw FFError("local execution: no weight named " + name);
  auto& t = val_[{it->second, 0}];
  if (static_cast<int64_t>(data.size()) != t.numel()) throw FFError("local execution: weight " + name + " size mismatch");
  t.v = data;
}
std::vector<float> LocalTrainingBacking::get_weight(const std::string& name) const {
  auto it = weight_of_.find(name);
  if (it == weight_of_.end()) throw FFError("local execution: no weight named " + name);
  return val_.at({it->second, 0}).v;
}
std::vector<float> LocalTrainingBacking::get_output() const { return val_.at(output_).v; }

HostTensor* LocalTrainingBacking::slot(const ValueRef& v, bool grad) {
  auto& m = grad ? grad_ : val_;
  auto it = m.find(v);
  return it == m.end() ? nullptr : &it->second;
}

void LocalTrainingBacking::forward_layer(int n) {
  const auto& node = cg_.g.node(n);
  auto it = registry().find(node.label.op.type);
  if (it == registry().end()) throw FFError("local execution: layer " + node.label.name + " is not an operator");
  OpCtx c;
  c.op = &node.label.op;
  for (auto const& v : cg_.layer_data_inputs(n)) c.in.push_back(&val_[v]);
  for (auto const& v : cg_.layer_weights(n)) c.w.push_back(&val_[v]);
  for (size_t i = 0; i < node.outputs.size(); ++i) c.out.push_back(&val_[{n, static_cast<int>(i)}]);
  c.saved = &saved_[n];
  c.training = true;
  c.seed = seed_ * 7919ull + static_cast<uint64_t>(n) * 104729ull + static_cast<uint64_t>(step_);
  const auto t0 = std::chrono::steady_clock::now();
  it->second.fwd(c);
  times_[n].first += elapsed_ms(t0);
}

void LocalTrainingBacking::forward() {
  for (int n : order_) forward_layer(n);
}

void LocalTrainingBacking::backward(const std::vector<float>& labels) {
  for (auto& kv : grad_) std::fill(kv.second.v.begin(), kv.second.v.end(), 0.f);
  const HostTensor& out = val_[output_];
  const int64_t C = out.dims.empty() ? 1 : out.dims.back();
  const int64_t R = out.numel() / C;
  // samples = leading (batch) dim; the reference scales every loss gradient by 1/batch
  const int64_t B = out.dims.empty() ? 1 : out.dims[0];
  const float scale = 1.f / static_cast<float>(std::max<int64_t>(R, 1));
  metrics_.samples += R;
  (void)B;
  if (loss_ == "sparse_categorical_crossentropy" || loss_ == "categorical_crossentropy") {
    const bool sparse = loss_ == "sparse_categorical_crossentropy";
    if (static_cast<int64_t>(labels.size()) != (sparse ? R : R * C))
      throw FFError("local execution: label size mismatch");
    // probabilities: the softmax output when fused, else softmax of the output
    std::vector<float> p(out.v);
    if (!fused_softmax_ce_) {
      for (int64_t r = 0; r < R; ++r) {
        float* pr = p.data() + r * C;
        const float m = *std::max_element(pr, pr + C);
        double s = 0;
        for (int64_t j = 0; j < C; ++j) s += (pr[j] = std::exp(pr[j] - m));
        for (int64_t j = 0; j < C; ++j) pr[j] = static_cast<float>(pr[j] / s);
      }
    }
    std::vector<float> g(p.size());
    for (int64_t r = 0; r < R; ++r) {
      const float* pr = p.data() + r * C;
      const int64_t am = std::max_element(pr, pr + C) - pr;
      if (sparse) {
        const int64_t y = static_cast<int64_t>(labels[r]);
        metrics_.loss_sum += -std::log(std::max(pr[y], 1e-30f));
        metrics_.correct += am == y;
        for (int64_t j = 0; j < C; ++j) g[r * C + j] = (pr[j] - (j == y ? 1.f : 0.f)) * scale;
      } else {
        const float* yr = labels.data() + r * C;
        double l = 0;
        for (int64_t j = 0; j < C; ++j) {
          l -= yr[j] * std::log(std::max(pr[j], 1e-30f));
          g[r * C + j] = (pr[j] - yr[j]) * scale;
        }
        metrics_.loss_sum += l;
        metrics_.correct += am == (std::max_element(yr, yr + C) - yr);
      }
    }
    // gradient w.r.t. the logits: the softmax input when fused
    const ValueRef tgt = fused_softmax_ce_ ? cg_.layer_data_inputs(output_.node)[0] : output_;
    if (grad_.count(tgt)) add_into(&grad_[tgt], g);
  } else if (loss_ == "mean_squared_error" || loss_ == "mean_squared_error_avg_reduce") {
    if (static_cast<int64_t>(labels.size()) != out.numel()) throw FFError("local execution: label size mismatch");
    std::vector<float> g(out.v.size());
    const float s = 2.f / static_cast<float>(R * C);
    double l = 0;
    for (size_t i = 0; i < g.size(); ++i) {
      const float d = out.v[i] - labels[i];
      l += d * d;
      g[i] = d * s;
    }
    metrics_.loss_sum += l / static_cast<double>(C);
    if (grad_.count(output_)) add_into(&grad_[output_], g);
  } else {  // identity
    metrics_.loss_sum += std::accumulate(out.v.begin(), out.v.end(), 0.0);
    if (grad_.count(output_)) add_into(&grad_[output_], std::vector<float>(out.v.size(), scale));
  }
  const auto& reg = registry();
  for (auto it = order_.rbegin(); it != order_.rend(); ++it) {
    const int n = *it;
    if (fused_softmax_ce_ && n == output_.node) continue;
    const auto& node = cg_.g.node(n);
    if (!needs_grad_[{n, 0}]) continue;
    OpCtx c;
    c.op = &node.label.op;
    for (auto const& v : cg_.layer_data_inputs(n)) {
      c.in.push_back(&val_[v]);
      c.d_in.push_back(grad_.count(v) ? &grad_[v] : nullptr);
    }
    for (auto const& v : cg_.layer_weights(n)) {
      c.w.push_back(&val_[v]);
      c.d_w.push_back(grad_.count(v) ? &grad_[v] : nullptr);
    }
    for (size_t i = 0; i < node.outputs.size(); ++i) {
      ValueRef v{n, static_cast<int>(i)};
      c.out.push_back(&val_[v]);
      c.d_out.push_back(&grad_[v]);
    }
    c.saved = &saved_[n];
    c.training = true;
    c.seed = seed_ * 7919ull + static_cast<uint64_t>(n) * 104729ull + static_cast<uint64_t>(step_);
    const auto t0 = std::chrono::steady_clock::now();
    reg.at(node.label.op.type).bwd(c);
    times_[n].second += elapsed_ms(t0);
  }
}

void LocalTrainingBacking::update() {
  ++step_;
  for (auto const& kv : weight_of_) {
    const int n = kv.second;
    const ValueRef v{n, 0};
    if (!grad_.count(v)) continue;
    auto& w = val_[v].v;
    const auto& g0 = grad_[v].v;
    const float lr = static_cast<float>(opt_.lr), wd = static_cast<float>(opt_.weight_decay);
    if (opt_.kind == "adam") {
      auto& m = m1_[n].v;
      auto& s = m2_[n].v;
      if (m.empty()) {
        m.assign(w.size(), 0.f);
        s.assign(w.size(), 0.f);
      }
      const float b1 = static_cast<float>(opt_.beta1), b2 = static_cast<float>(opt_.beta2);
      const float bc1 = 1.f - static_cast<float>(std::pow(opt_.beta1, static_cast<double>(step_)));
      const float bc2 = 1.f - static_cast<float>(std::pow(opt_.beta2, static_cast<double>(step_)));
      for (size_t i = 0; i < w.size(); ++i) {
        const float g = g0[i] + wd * w[i];  // L2 folded into the gradient (reference adam_update)
        m[i] = b1 * m[i] + (1.f - b1) * g;
        s[i] = b2 * s[i] + (1.f - b2) * g * g;
        w[i] -= lr * (m[i] / bc1) / (std::sqrt(s[i] / bc2) + static_cast<float>(opt_.epsilon));
      }
    } else {
      const float mom = static_cast<float>(opt_.momentum);
      auto& buf = m1_[n].v;
      if (mom != 0.f && buf.empty()) buf.assign(w.size(), 0.f);
      for (size_t i = 0; i < w.size(); ++i) {
        float g = g0[i] + wd * w[i];
        if (mom != 0.f) {
          buf[i] = mom * buf[i] + g;
          g = opt_.nesterov ? g + mom * buf[i] : buf[i];
        }
        w[i] -= lr * g;
      }
    }
  }
}

std::map<std::string, std::pair<double, double>> LocalTrainingBacking::layer_times_ms() const {
  std::map<std::string, std::pair<double, double>> r;
  for (auto const& kv : times_) r[cg_.g.node(kv.first).label.name] = kv.second;
  return r;
}

// ---------------------------------------------------------------------------
double measure_op_cost_ms(const OpAttrs& op, const std::vector<TensorShape>& input_shapes, int iters) {
  ComputationGraph cg;
  std::vector<ValueRef> ins;
  for (size_t i = 0; i < input_shapes.size(); ++i)
    ins.push_back(cg.create_input(input_shapes[i], true, "in" + std::to_string(i)));
  auto outs = cg.add_layer(op, ins, "op");
  LocalOptimizer o;
  o.lr = 0.0;
  LocalTrainingBacking b(cg, o, "identity", 1, /*input_grads=*/true);
  std::mt19937 rng(0);
  std::uniform_real_distribution<float> d(0.f, 1.f);
  for (size_t i = 0; i < ins.size(); ++i) {
    std::vector<float> x(static_cast<size_t>(input_shapes[i].num_elements()));
    for (auto& e : x) e = d(rng);
    b.set_input("in" + std::to_string(i), x);
  }
  std::vector<double> t;
  for (int it = 0; it <= std::max(1, iters); ++it) {
    const auto t0 = std::chrono::steady_clock::now();
    b.forward();
    b.backward({});
    if (it > 0) t.push_back(elapsed_ms(t0));  // first run = warm-up
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

}  // namespace ff
