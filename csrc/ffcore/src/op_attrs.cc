#include "ff/op_attrs.h"

#include <algorithm>
#include <functional>
#include <numeric>
#include <sstream>
#include <unordered_map>

namespace ff {

// ---------------------------------------------------------------------------
// AttrValue helpers
Json attr_to_json(const AttrValue& v) {
  switch (v.index()) {
    case 0: return Json(std::get<int64_t>(v));
    case 1: {
      Json j = Json::object();
      j["f"] = std::get<double>(v);
      return j;
    }
    case 2: return Json(std::get<bool>(v));
    case 3: return Json(std::get<std::string>(v));
    default: {
      Json j = Json::object();
      j["ints"] = Json(std::get<std::vector<int64_t>>(v));
      return j;
    }
  }
}

AttrValue attr_from_json(const Json& j) {
  if (j.is_bool()) return j.as_bool();
  if (j.is_int()) return j.as_int();
  if (j.is_number()) return j.as_double();
  if (j.is_string()) return j.as_string();
  if (j.is_object() && j.contains("f")) return j.at("f").as_double();
  if (j.is_object() && j.contains("ints")) return j.at("ints").as_int_vector();
  if (j.is_array()) return j.as_int_vector();
  throw FFError("attr_from_json: unsupported value " + j.dump());
}

std::string attr_to_string(const AttrValue& v) {
  std::ostringstream os;
  switch (v.index()) {
    case 0: os << std::get<int64_t>(v); break;
    case 1: os << std::get<double>(v); break;
    case 2: os << (std::get<bool>(v) ? "true" : "false"); break;
    case 3: os << std::get<std::string>(v); break;
    default: {
      auto const& xs = std::get<std::vector<int64_t>>(v);
      os << "[";
      for (size_t i = 0; i < xs.size(); ++i) os << (i ? "," : "") << xs[i];
      os << "]";
    }
  }
  return os.str();
}

int64_t OpAttrs::i(const std::string& k) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) throw FFError(to_string(type) + ": missing int attr " + k);
  if (auto p = std::get_if<int64_t>(&it->second)) return *p;
  if (auto p = std::get_if<bool>(&it->second)) return *p ? 1 : 0;
  if (auto p = std::get_if<double>(&it->second)) return static_cast<int64_t>(*p);
  throw FFError(to_string(type) + ": attr " + k + " is not an int");
}
double OpAttrs::f(const std::string& k) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) throw FFError(to_string(type) + ": missing float attr " + k);
  if (auto p = std::get_if<double>(&it->second)) return *p;
  if (auto p = std::get_if<int64_t>(&it->second)) return static_cast<double>(*p);
  throw FFError(to_string(type) + ": attr " + k + " is not a float");
}
bool OpAttrs::b(const std::string& k) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) throw FFError(to_string(type) + ": missing bool attr " + k);
  if (auto p = std::get_if<bool>(&it->second)) return *p;
  if (auto p = std::get_if<int64_t>(&it->second)) return *p != 0;
  throw FFError(to_string(type) + ": attr " + k + " is not a bool");
}
const std::string& OpAttrs::s(const std::string& k) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) throw FFError(to_string(type) + ": missing string attr " + k);
  if (auto p = std::get_if<std::string>(&it->second)) return *p;
  throw FFError(to_string(type) + ": attr " + k + " is not a string");
}
const std::vector<int64_t>& OpAttrs::ints(const std::string& k) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) throw FFError(to_string(type) + ": missing list attr " + k);
  if (auto p = std::get_if<std::vector<int64_t>>(&it->second)) return *p;
  throw FFError(to_string(type) + ": attr " + k + " is not a list");
}

size_t OpAttrs::hash() const {
  size_t h = std::hash<int>()(static_cast<int>(type));
  for (auto const& kv : attrs) {
    h = hash_combine(h, std::hash<std::string>()(kv.first));
    h = hash_combine(h, std::hash<std::string>()(attr_to_string(kv.second)));
  }
  return h;
}

std::string OpAttrs::str() const {
  std::ostringstream os;
  os << to_string(type) << "(";
  bool first = true;
  for (auto const& kv : attrs) {
    os << (first ? "" : ", ") << kv.first << "=" << attr_to_string(kv.second);
    first = false;
  }
  os << ")";
  return os.str();
}

Json OpAttrs::to_json() const {
  Json j = Json::object();
  j["op_type"] = to_string(type);
  Json a = Json::object();
  for (auto const& kv : attrs) a[kv.first] = attr_to_json(kv.second);
  j["attrs"] = a;
  return j;
}

OpAttrs OpAttrs::from_json(const Json& j) {
  OpAttrs a(optype_from_string(j.at("op_type").as_string()));
  if (j.contains("attrs"))
    for (auto const& kv : j.at("attrs").as_object()) a.attrs[kv.first] = attr_from_json(kv.second);
  return a;
}

// ---------------------------------------------------------------------------
// Registry
namespace {

using Shapes = std::vector<TensorShape>;
using PShapes = std::vector<ParallelTensorShape>;
using SerialFn = std::function<Shapes(const OpAttrs&, const Shapes&)>;
using ParFn = std::function<PShapes(const OpAttrs&, const PShapes&)>;

struct OpSpec {
  int num_inputs = 1;  // -1 variadic
  std::map<std::string, AttrValue> defaults;
  std::vector<std::string> required;
  std::function<std::vector<std::string>(const OpAttrs&)> weights;
  SerialFn out;
  SerialFn wts;
  ParFn pout;
  ParFn pwts;
};

[[noreturn]] void bad(const OpAttrs& a, const std::string& msg) {
  throw FFError(to_string(a.type) + ": " + msg);
}

void require(bool cond, const OpAttrs& a, const std::string& msg) {
  if (!cond) bad(a, msg);
}

std::vector<std::string> no_weights(const OpAttrs&) { return {}; }
Shapes no_weight_shapes(const OpAttrs&, const Shapes&) { return {}; }
PShapes no_pweight_shapes(const OpAttrs&, const PShapes&) { return {}; }

// Elementwise ops that are linear in their input commute with a pending
// partial sum; nonlinear ones do not.
bool is_linear_unary(OpType t) {
  return t == OpType::IDENTITY || t == OpType::SCALAR_MULTIPLY || t == OpType::SCALAR_TRUE_DIV ||
         t == OpType::NOOP;
}

int nd(const TensorShape& s) { return s.num_dims(); }

std::vector<int64_t> broadcast_dims(const OpAttrs& a, std::vector<int64_t> x, std::vector<int64_t> y) {
  size_t n = std::max(x.size(), y.size());
  x.insert(x.begin(), n - x.size(), 1);
  y.insert(y.begin(), n - y.size(), 1);
  std::vector<int64_t> r(n);
  for (size_t i = 0; i < n; ++i) {
    if (x[i] == y[i] || y[i] == 1) r[i] = x[i];
    else if (x[i] == 1) r[i] = y[i];
    else bad(a, "shapes not broadcastable");
  }
  return r;
}

int64_t conv_out(int64_t in, int64_t k, int64_t s, int64_t p) { return (in + 2 * p - k) / s + 1; }

// Attribute (spatial) parallelism of a window op along H (flexflow_train_amd/
// parallel/halo.py): shard j of d computes output rows [j OH/d, (j+1) OH/d)
// from its input rows plus halos taken from its two neighbours; every shard's
// halo must fit inside one neighbour's rows.
bool spatial_split_ok(int64_t H, int64_t k, int64_t s, int64_t p, int d) {
  if (d <= 1) return true;
  const int64_t OH = conv_out(H, k, s, p);
  if (H % d || OH % d || OH <= 0) return false;
  const int64_t Hl = H / d, OHl = OH / d;
  for (int j = 0; j < d; ++j) {
    const int64_t lo = j * OHl * s - p, hi = ((j + 1) * OHl - 1) * s - p + k;
    const int64_t top = std::max<int64_t>(0, j * Hl - std::max<int64_t>(lo, 0));
    const int64_t bot = std::max<int64_t>(0, std::min<int64_t>(hi, H) - (j + 1) * Hl);
    if (top > Hl || bot > Hl) return false;
    if ((j == 0 && top) || (j == d - 1 && bot)) return false;
  }
  return true;
}

std::vector<int> norm_axes(const OpAttrs& a, const std::string& key, int ndims) {
  std::vector<int> r;
  for (auto x : a.ints(key)) r.push_back(normalize_dim(static_cast<int>(x), ndims));
  std::sort(r.begin(), r.end());
  return r;
}

std::unordered_map<int, OpSpec>& registry();

}  // namespace

// ---------------------------------------------------------------------------
namespace {

OpSpec unary_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.weights = no_weights;
  s.out = [](const OpAttrs&, const Shapes& in) { return Shapes{in.at(0)}; };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    if (!is_linear_unary(a.type) && in.at(0).sum_degree != 1)
      bad(a, "nonlinear elementwise op applied to a partial-sum tensor");
    return PShapes{in.at(0)};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec binary_spec() {
  OpSpec s;
  s.num_inputs = 2;
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    TensorShape o;
    o.dtype = in.at(0).dtype;
    o.dims = broadcast_dims(a, in.at(0).dims, in.at(1).dims);
    if (a.type == OpType::EW_EQUAL || a.type == OpType::EW_GREATER || a.type == OpType::EW_LESS)
      o.dtype = DataType::BOOL;
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto x = in.at(0), y = in.at(1);
    size_t n = std::max(x.shard_dims.size(), y.shard_dims.size());
    x.shard_dims.insert(x.shard_dims.begin(), n - x.shard_dims.size(), ShardParallelDim{1, 1});
    y.shard_dims.insert(y.shard_dims.begin(), n - y.shard_dims.size(), ShardParallelDim{1, 1});
    ParallelTensorShape o = x;
    for (size_t i = 0; i < n; ++i) {
      auto dx = x.shard_dims[i], dy = y.shard_dims[i];
      if (dx.size == dy.size) {
        require(dx.degree == dy.degree, a, "operand shard degrees differ on dim " + std::to_string(i));
        o.shard_dims[i] = dx;
      } else if (dx.size == 1) {
        require(dx.degree == 1, a, "broadcast dim must be unpartitioned");
        o.shard_dims[i] = dy;
      } else {
        require(dy.degree == 1, a, "broadcast dim must be unpartitioned");
        o.shard_dims[i] = dx;
      }
    }
    if (a.type == OpType::EW_ADD || a.type == OpType::EW_SUB) {
      require(x.sum_degree == y.sum_degree, a, "operands have different partial-sum degrees");
    } else {
      require(x.sum_degree == 1 && y.sum_degree == 1, a, "nonlinear binary op on partial sums");
    }
    require(x.total_parallel_degree() == y.total_parallel_degree(), a,
            "operands have different total parallel degree");
    o.sum_degree = x.sum_degree;
    int shard = static_cast<int>(product(o.shard_degrees()));
    o.discard_copy_degree = x.total_parallel_degree() / (shard * o.sum_degree);
    require(o.total_parallel_degree() == x.total_parallel_degree(), a, "inconsistent degrees");
    if (a.type == OpType::EW_EQUAL || a.type == OpType::EW_GREATER || a.type == OpType::EW_LESS)
      o.dtype = DataType::BOOL;
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec linear_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"out_channels"};
  s.defaults = {{"use_bias", true}, {"activation", std::string("none")},
                {"regularizer", std::string("none")}, {"regularizer_lambda", 0.0}};
  s.weights = [](const OpAttrs& a) {
    std::vector<std::string> w{"kernel"};
    if (a.b("use_bias")) w.push_back("bias");
    return w;
  };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    TensorShape o = in.at(0);
    require(nd(o) >= 1, a, "input must have rank >= 1");
    o.at(-1) = a.i("out_channels");
    return Shapes{o};
  };
  s.wts = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in.at(0);
    Shapes w{TensorShape{{x.at(-1), a.i("out_channels")}, x.dtype}};
    if (a.b("use_bias")) w.push_back(TensorShape{{a.i("out_channels")}, x.dtype});
    return w;
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    if (activation_from_string(a.s("activation")) != Activation::NONE)
      require(x.dim(-1).degree == 1 && x.sum_degree == 1, a,
              "fused activation requires a complete (non partial-sum) output");
    TensorShape o = registry()[static_cast<int>(OpType::LINEAR)].out(a, {x.reduced_shape()})[0];
    std::vector<int> deg = x.shard_degrees();
    deg.back() = x.discard_copy_degree;
    return PShapes{lift_to_parallel_with_degrees(o, x.sum_degree * x.dim(-1).degree, 1, deg)};
  };
  s.pwts = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    auto ws = registry()[static_cast<int>(OpType::LINEAR)].wts(a, {x.reduced_shape()});
    auto deg = x.shard_degrees();
    int non_last = static_cast<int>(product(std::vector<int>(deg.begin(), deg.end() - 1)));
    PShapes r{lift_to_parallel_with_degrees(ws[0], 1, x.sum_degree * non_last,
                                            {x.dim(-1).degree, x.discard_copy_degree})};
    if (ws.size() > 1)
      r.push_back(lift_to_parallel_with_degrees(ws[1], x.sum_degree * x.dim(-1).degree, non_last,
                                                {x.discard_copy_degree}));
    return r;
  };
  return s;
}

OpSpec conv2d_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"out_channels", "kernel_h", "kernel_w"};
  s.defaults = {{"stride_h", int64_t(1)}, {"stride_w", int64_t(1)}, {"padding_h", int64_t(0)},
                {"padding_w", int64_t(0)}, {"groups", int64_t(1)},
                {"activation", std::string("none")}, {"use_bias", true}};
  s.weights = [](const OpAttrs& a) {
    std::vector<std::string> w{"kernel"};
    if (a.b("use_bias")) w.push_back("bias");
    return w;
  };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in.at(0);
    require(nd(x) == 4, a, "input must be NCHW");
    require(x.dims[1] % a.i("groups") == 0, a, "channels not divisible by groups");
    TensorShape o{{x.dims[0], a.i("out_channels"),
                   conv_out(x.dims[2], a.i("kernel_h"), a.i("stride_h"), a.i("padding_h")),
                   conv_out(x.dims[3], a.i("kernel_w"), a.i("stride_w"), a.i("padding_w"))},
                  x.dtype};
    return Shapes{o};
  };
  s.wts = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in.at(0);
    Shapes w{TensorShape{{a.i("out_channels"), x.dims[1] / a.i("groups"), a.i("kernel_h"), a.i("kernel_w")},
                         x.dtype}};
    if (a.b("use_bias")) w.push_back(TensorShape{{a.i("out_channels")}, x.dtype});
    return w;
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    // attribute parallelism: H shards with halo exchange (W stays whole)
    const int dh = x.dim(2).degree;
    require(x.dim(3).degree == 1, a, "W (attribute) degree must be 1");
    require(dh == 1 || spatial_split_ok(x.dim(2).size, a.i("kernel_h"), a.i("stride_h"), a.i("padding_h"), dh), a,
            "H shards need halos wider than one neighbour");
    require(a.i("groups") == 1 || x.dim(1).degree == 1, a, "grouped conv cannot shard channels");
    if (activation_from_string(a.s("activation")) != Activation::NONE)
      require(x.dim(1).degree == 1 && x.sum_degree == 1, a, "fused activation on partial sums");
    auto o = registry()[static_cast<int>(OpType::CONV2D)].out(a, {x.reduced_shape()})[0];
    return PShapes{lift_to_parallel_with_degrees(o, x.sum_degree * x.dim(1).degree, 1,
                                                 {x.dim(0).degree, x.discard_copy_degree, dh, 1})};
  };
  s.pwts = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    const int dh = x.dim(2).degree;
    auto ws = registry()[static_cast<int>(OpType::CONV2D)].wts(a, {x.reduced_shape()});
    PShapes r{lift_to_parallel_with_degrees(ws[0], 1, x.dim(0).degree * dh * x.sum_degree,
                                            {x.discard_copy_degree, x.dim(1).degree, 1, 1})};
    if (ws.size() > 1)
      r.push_back(lift_to_parallel_with_degrees(ws[1], x.sum_degree * x.dim(1).degree, x.dim(0).degree * dh,
                                                {x.discard_copy_degree}));
    return r;
  };
  return s;
}

OpSpec pool2d_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"kernel_h", "kernel_w"};
  s.defaults = {{"stride_h", int64_t(1)}, {"stride_w", int64_t(1)}, {"padding_h", int64_t(0)},
                {"padding_w", int64_t(0)}, {"pool_type", std::string("max")},
                {"activation", std::string("none")}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in.at(0);
    require(nd(x) == 4, a, "input must be NCHW");
    return Shapes{TensorShape{{x.dims[0], x.dims[1],
                               conv_out(x.dims[2], a.i("kernel_h"), a.i("stride_h"), a.i("padding_h")),
                               conv_out(x.dims[3], a.i("kernel_w"), a.i("stride_w"), a.i("padding_w"))},
                              x.dtype}};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    const int dh = x.dim(2).degree;
    require(x.dim(3).degree == 1, a, "W (attribute) degree must be 1");
    require(dh == 1 || spatial_split_ok(x.dim(2).size, a.i("kernel_h"), a.i("stride_h"), a.i("padding_h"), dh), a,
            "H shards need halos wider than one neighbour");
    // average pooling without an activation is linear: partial sums pass
    // through (pool_2d.cc "PoolOp::AVG does allow sum parallelism")
    const bool linear = a.s("pool_type") == "avg" && a.s("activation") == "none";
    require(x.sum_degree == 1 || linear, a, "pooling a partial-sum tensor");
    auto o = registry()[static_cast<int>(OpType::POOL2D)].out(a, {x.reduced_shape()})[0];
    return PShapes{lift_to_parallel_with_degrees(o, x.sum_degree, x.discard_copy_degree,
                                                 {x.dim(0).degree, x.dim(1).degree, dh, 1})};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec batchnorm_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.defaults = {{"relu", false}, {"affine", true}, {"eps", 1e-5}, {"momentum", 0.1}};
  s.weights = [](const OpAttrs& a) {
    return a.b("affine") ? std::vector<std::string>{"gamma", "beta"} : std::vector<std::string>{};
  };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    require(nd(in.at(0)) >= 2, a, "input must have a channel dim");
    return Shapes{in.at(0)};
  };
  s.wts = [](const OpAttrs& a, const Shapes& in) {
    if (!a.b("affine")) return Shapes{};
    TensorShape w{{in.at(0).dims[1]}, in.at(0).dtype};
    return Shapes{w, w};
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    require(x.sum_degree == 1, a, "normalizing a partial-sum tensor");
    // spatial (H / W) degrees must be 1, as in the reference
    // (lib/op-attrs/src/op-attrs/ops/batch_norm.cc): a band would normalise
    // with its own statistics and change what the model computes, so the
    // search has to Combine the bands before a BatchNorm.  Batch shards keep
    // per-device statistics (the reference's data-parallel BatchNorm).
    for (int d = 2; d < x.num_dims(); ++d) require(x.dim(d).degree == 1, a, "spatial degrees must be 1");
    return PShapes{x};
  };
  s.pwts = [](const OpAttrs& a, const PShapes& in) {
    if (!a.b("affine")) return PShapes{};
    auto const& x = in.at(0);
    auto w = lift_to_parallel_with_degrees(TensorShape{{x.dim(1).size}, x.dtype}, 1,
                                           x.dim(0).degree * x.discard_copy_degree, {x.dim(1).degree});
    return PShapes{w, w};
  };
  return s;
}

OpSpec layernorm_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.defaults = {{"axes", std::vector<int64_t>{-1}}, {"elementwise_affine", true}, {"eps", 1e-5},
                {"use_bias", true}};
  s.weights = [](const OpAttrs& a) {
    if (!a.b("elementwise_affine")) return std::vector<std::string>{};
    if (!a.b("use_bias")) return std::vector<std::string>{"gamma"};
    return std::vector<std::string>{"gamma", "beta"};
  };
  s.out = [](const OpAttrs&, const Shapes& in) { return Shapes{in.at(0)}; };
  s.wts = [](const OpAttrs& a, const Shapes& in) {
    if (!a.b("elementwise_affine")) return Shapes{};
    TensorShape w{{}, in.at(0).dtype};
    for (int ax : norm_axes(a, "axes", nd(in.at(0)))) w.dims.push_back(in.at(0).dims[ax]);
    return a.b("use_bias") ? Shapes{w, w} : Shapes{w};
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    require(x.sum_degree == 1, a, "normalizing a partial-sum tensor");
    for (int ax : norm_axes(a, "axes", x.num_dims()))
      require(x.shard_dims[ax].degree == 1, a, "normalized axis must be unpartitioned");
    return PShapes{x};
  };
  s.pwts = [](const OpAttrs& a, const PShapes& in) {
    if (!a.b("elementwise_affine")) return PShapes{};
    auto const& x = in.at(0);
    TensorShape w{{}, x.dtype};
    std::vector<int> deg;
    auto axes = norm_axes(a, "axes", x.num_dims());
    int other = 1;
    for (int d = 0; d < x.num_dims(); ++d) {
      if (std::find(axes.begin(), axes.end(), d) != axes.end()) {
        w.dims.push_back(x.shard_dims[d].size);
        deg.push_back(1);
      } else {
        other *= x.shard_dims[d].degree;
      }
    }
    auto pw = lift_to_parallel_with_degrees(w, 1, other * x.discard_copy_degree, deg);
    return a.b("use_bias") ? PShapes{pw, pw} : PShapes{pw};
  };
  return s;
}

OpSpec softmax_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.defaults = {{"dim", int64_t(-1)}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    normalize_dim(static_cast<int>(a.i("dim")), nd(in.at(0)));
    return Shapes{in.at(0)};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    require(x.sum_degree == 1, a, "softmax of a partial-sum tensor");
    require(x.dim(static_cast<int>(a.i("dim"))).degree == 1, a, "softmax dim must be unpartitioned");
    return PShapes{x};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec embedding_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"num_entries", "out_channels"};
  s.defaults = {{"aggr", std::string("none")}, {"data_type", std::string("float")}};
  s.weights = [](const OpAttrs&) { return std::vector<std::string>{"weight"}; };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in.at(0);
    TensorShape o;
    o.dtype = datatype_from_string(a.s("data_type"));
    o.dims = x.dims;
    if (a.s("aggr") == "none") {
      o.dims.push_back(a.i("out_channels"));
    } else {
      require(nd(x) >= 1, a, "bag input needs rank >= 1");
      o.dims.back() = a.i("out_channels");
    }
    return Shapes{o};
  };
  s.wts = [](const OpAttrs& a, const Shapes&) {
    return Shapes{TensorShape{{a.i("num_entries"), a.i("out_channels")},
                              datatype_from_string(a.s("data_type"))}};
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    require(x.sum_degree == 1, a, "indices cannot be partial sums");
    auto o = registry()[static_cast<int>(OpType::EMBEDDING)].out(a, {x.reduced_shape()})[0];
    auto deg = x.shard_degrees();
    int sum = 1;
    if (a.s("aggr") == "none") {
      deg.push_back(x.discard_copy_degree);
    } else {
      sum = deg.back();
      deg.back() = x.discard_copy_degree;
    }
    return PShapes{lift_to_parallel_with_degrees(o, sum, 1, deg)};
  };
  s.pwts = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in.at(0);
    auto w = registry()[static_cast<int>(OpType::EMBEDDING)].wts(a, {x.reduced_shape()})[0];
    return PShapes{lift_to_parallel_with_degrees(w, 1, static_cast<int>(product(x.shard_degrees())),
                                                 {1, x.discard_copy_degree})};
  };
  return s;
}

// Multi-head attention.  Inputs q,k,v: [batch, seq, features].
// Weight: [qSize*kdim + kSize*kdim + vSize*vdim + vdim*embed_dim, num_heads]
// (ops/attention.cc:136-170); input bias [2*kdim + vdim, num_heads],
// output bias [embed_dim].
OpSpec mha_spec() {
  OpSpec s;
  s.num_inputs = 3;
  s.required = {"embed_dim", "num_heads"};
  s.defaults = {{"kdim", int64_t(0)}, {"vdim", int64_t(0)}, {"dropout", 0.0}, {"bias", true},
                {"add_bias_kv", false}, {"add_zero_attn", false}, {"causal", false},
                {"seq_parallel_mode", std::string("auto")}};  // auto | ulysses | ring
  s.weights = [](const OpAttrs& a) {
    std::vector<std::string> w{"weight"};
    if (a.b("bias")) {
      w.push_back("input_bias");
      w.push_back("output_bias");
    }
    return w;
  };
  auto kd = [](const OpAttrs& a) {
    return a.i("kdim") > 0 ? a.i("kdim") : a.i("embed_dim") / a.i("num_heads");
  };
  auto vd = [](const OpAttrs& a) {
    return a.i("vdim") > 0 ? a.i("vdim") : a.i("embed_dim") / a.i("num_heads");
  };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    for (auto const& t : in) require(nd(t) == 3, a, "q/k/v must be [batch, seq, feature]");
    require(in[0].dims[0] == in[1].dims[0] && in[0].dims[0] == in[2].dims[0], a, "batch mismatch");
    require(in[1].dims[1] == in[2].dims[1], a, "key/value sequence length mismatch");
    return Shapes{TensorShape{{in[0].dims[0], in[0].dims[1], a.i("embed_dim")}, in[0].dtype}};
  };
  s.wts = [kd, vd](const OpAttrs& a, const Shapes& in) {
    int64_t k = kd(a), v = vd(a);
    int64_t p = in[0].dims[2] * k + in[1].dims[2] * k + in[2].dims[2] * v + v * a.i("embed_dim");
    Shapes w{TensorShape{{p, a.i("num_heads")}, in[0].dtype}};
    if (a.b("bias")) {
      w.push_back(TensorShape{{2 * k + v, a.i("num_heads")}, in[0].dtype});
      w.push_back(TensorShape{{a.i("embed_dim")}, in[0].dtype});
    }
    return w;
  };
  auto parse = [](const OpAttrs& a, const PShapes& in) {
    for (auto const& t : in) {
      require(t.num_dims() == 3, a, "q/k/v must be rank 3");
      require(t.sum_degree == 1, a, "attention inputs cannot be partial sums");
      require(t.dim(2).degree == 1, a, "feature dim must be unpartitioned");
    }
    require(in[0].dim(0).degree == in[1].dim(0).degree && in[0].dim(0).degree == in[2].dim(0).degree,
            a, "q/k/v batch degrees differ");
    require(in[0].discard_copy_degree == in[1].discard_copy_degree &&
                in[0].discard_copy_degree == in[2].discard_copy_degree,
            a, "q/k/v replica degrees differ");
    require(in[1].dim(1).degree == in[2].dim(1).degree, a, "k/v sequence degrees differ");
    // Sequence (context) parallelism: q may be sharded on seq; k/v must carry
    // the same degree (ring / all-to-all lowering in the runtime).
    require(in[0].dim(1).degree == in[1].dim(1).degree, a, "q/kv sequence degrees differ");
    require(a.i("num_heads") % in[0].discard_copy_degree == 0, a, "heads not divisible by head degree");
  };
  s.pout = [parse](const OpAttrs& a, const PShapes& in) {
    parse(a, in);
    auto o = registry()[static_cast<int>(OpType::MULTIHEAD_ATTENTION)].out(
        a, {in[0].reduced_shape(), in[1].reduced_shape(), in[2].reduced_shape()})[0];
    return PShapes{lift_to_parallel_with_degrees(o, in[0].discard_copy_degree, 1,
                                                 {in[0].dim(0).degree, in[0].dim(1).degree, 1})};
  };
  s.pwts = [parse](const OpAttrs& a, const PShapes& in) {
    parse(a, in);
    auto ws = registry()[static_cast<int>(OpType::MULTIHEAD_ATTENTION)].wts(
        a, {in[0].reduced_shape(), in[1].reduced_shape(), in[2].reduced_shape()});
    int dp = in[0].dim(0).degree * in[0].dim(1).degree;
    int hp = in[0].discard_copy_degree;
    PShapes r{lift_to_parallel_with_degrees(ws[0], 1, dp, {1, hp})};
    if (ws.size() > 1) {
      r.push_back(lift_to_parallel_with_degrees(ws[1], 1, dp, {1, hp}));
      r.push_back(lift_to_parallel_with_degrees(ws[2], hp, dp, {1}));
    }
    return r;
  };
  return s;
}

OpSpec batch_matmul_spec() {
  OpSpec s;
  s.num_inputs = 2;
  s.defaults = {{"a_seq_length_dim", int64_t(-1)}, {"b_seq_length_dim", int64_t(-1)}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const &x = in.at(0), &y = in.at(1);
    require(nd(x) >= 2 && nd(x) == nd(y), a, "operands must have equal rank >= 2");
    require(x.at(-1) == y.at(-2), a, "inner dims mismatch");
    for (int d = 0; d < nd(x) - 2; ++d) require(x.dims[d] == y.dims[d], a, "batch dims mismatch");
    TensorShape o = x;
    o.at(-1) = y.at(-1);
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const &x = in.at(0), &y = in.at(1);
    require(x.sum_degree == 1 && y.sum_degree == 1, a, "partial-sum operands");
    int n = x.num_dims();
    for (int d = 0; d < n - 2; ++d)
      require(x.shard_dims[d].degree == y.shard_dims[d].degree, a, "batch degrees differ");
    require(x.dim(-1).degree == y.dim(-2).degree, a, "reduction degrees differ");
    require(x.discard_copy_degree == y.dim(-1).degree, a, "lhs replicas must match rhs column shards");
    require(y.discard_copy_degree == x.dim(-2).degree, a, "rhs replicas must match lhs row shards");
    auto o = registry()[static_cast<int>(OpType::BATCHMATMUL)].out(a, {x.reduced_shape(), y.reduced_shape()})[0];
    auto deg = x.shard_degrees();
    deg[n - 1] = y.dim(-1).degree;
    return PShapes{lift_to_parallel_with_degrees(o, x.dim(-1).degree, 1, deg)};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec concat_spec() {
  OpSpec s;
  s.num_inputs = -1;
  s.required = {"axis"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    require(!in.empty(), a, "needs inputs");
    int ax = normalize_dim(static_cast<int>(a.i("axis")), nd(in[0]));
    TensorShape o = in[0];
    o.dims[ax] = 0;
    for (auto const& t : in) {
      require(nd(t) == nd(in[0]), a, "rank mismatch");
      for (int d = 0; d < nd(t); ++d)
        if (d != ax) require(t.dims[d] == in[0].dims[d], a, "non-axis dims mismatch");
      o.dims[ax] += t.dims[ax];
    }
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    int ax = normalize_dim(static_cast<int>(a.i("axis")), in[0].num_dims());
    for (auto const& t : in) {
      require(t.shard_dims[ax].degree == 1, a, "concat axis must be unpartitioned");
      require(t.shard_degrees() == in[0].shard_degrees() && t.sum_degree == in[0].sum_degree &&
                  t.discard_copy_degree == in[0].discard_copy_degree,
              a, "inputs have different parallel degrees");
    }
    ParallelTensorShape o = in[0];
    o.shard_dims[ax].size = 0;
    for (auto const& t : in) o.shard_dims[ax].size += t.shard_dims[ax].size;
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec split_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"axis", "splits"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    int ax = normalize_dim(static_cast<int>(a.i("axis")), nd(in[0]));
    auto const& sp = a.ints("splits");
    require(std::accumulate(sp.begin(), sp.end(), int64_t(0)) == in[0].dims[ax], a, "splits do not sum to dim");
    Shapes r;
    for (auto v : sp) {
      TensorShape o = in[0];
      o.dims[ax] = v;
      r.push_back(o);
    }
    return r;
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    int ax = normalize_dim(static_cast<int>(a.i("axis")), in[0].num_dims());
    require(in[0].shard_dims[ax].degree == 1, a, "split axis must be unpartitioned");
    PShapes r;
    for (auto v : a.ints("splits")) {
      auto o = in[0];
      o.shard_dims[ax].size = v;
      r.push_back(o);
    }
    return r;
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec flat_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.defaults = {{"start_dim", int64_t(1)}, {"end_dim", int64_t(-1)}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in[0];
    int st = normalize_dim(static_cast<int>(a.i("start_dim")), nd(x));
    int en = normalize_dim(static_cast<int>(a.i("end_dim")), nd(x));
    if (en < st) return Shapes{x};   // empty range: identity (flat.cc "flatten no dims")
    TensorShape o{{}, x.dtype};
    for (int d = 0; d < st; ++d) o.dims.push_back(x.dims[d]);
    int64_t p = 1;
    for (int d = st; d <= en; ++d) p *= x.dims[d];
    o.dims.push_back(p);
    for (int d = en + 1; d < nd(x); ++d) o.dims.push_back(x.dims[d]);
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in[0];
    int st = normalize_dim(static_cast<int>(a.i("start_dim")), x.num_dims());
    int en = normalize_dim(static_cast<int>(a.i("end_dim")), x.num_dims());
    if (en < st) return PShapes{x};
    for (int d = st + 1; d <= en; ++d) require(x.shard_dims[d].degree == 1, a, "flattened inner dims must be unpartitioned");
    auto o = registry()[static_cast<int>(OpType::FLAT)].out(a, {x.reduced_shape()})[0];
    std::vector<int> deg;
    for (int d = 0; d < st; ++d) deg.push_back(x.shard_dims[d].degree);
    deg.push_back(x.shard_dims[st].degree);
    for (int d = en + 1; d < x.num_dims(); ++d) deg.push_back(x.shard_dims[d].degree);
    return PShapes{lift_to_parallel_with_degrees(o, x.sum_degree, x.discard_copy_degree, deg)};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec reshape_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"shape"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& x = in[0];
    TensorShape o{{}, x.dtype};
    int64_t known = 1;
    int infer = -1;
    auto const& sh = a.ints("shape");
    for (size_t i = 0; i < sh.size(); ++i) {
      if (sh[i] == -1) {
        require(infer < 0, a, "at most one -1 in shape");
        infer = static_cast<int>(i);
        o.dims.push_back(1);
      } else {
        known *= sh[i];
        o.dims.push_back(sh[i]);
      }
    }
    if (infer >= 0) o.dims[infer] = x.num_elements() / known;
    require(o.num_elements() == x.num_elements(), a, "element count mismatch");
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in[0];
    auto o = registry()[static_cast<int>(OpType::RESHAPE)].out(a, {x.reduced_shape()})[0];
    std::vector<int> deg(o.dims.size(), 1);
    for (int d = 1; d < x.num_dims(); ++d) require(x.shard_dims[d].degree == 1, a, "only the outer dim may be partitioned");
    if (x.shard_dims[0].degree > 1) {
      require(o.dims[0] % x.shard_dims[0].degree == 0 && o.dims[0] * 1 > 0, a, "outer dim not divisible");
      // outer-dim sharding is preserved when the outer dim is a multiple of the old outer dim
      // or vice versa (the reshape keeps contiguous outer blocks).
      require(o.dims[0] % x.shard_dims[0].size == 0 || x.shard_dims[0].size % o.dims[0] == 0, a,
              "reshape does not preserve outer-dim blocks");
      deg[0] = x.shard_dims[0].degree;
    }
    return PShapes{lift_to_parallel_with_degrees(o, x.sum_degree, x.discard_copy_degree, deg)};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec transpose_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"perm"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto const& p = a.ints("perm");
    require(static_cast<int>(p.size()) == nd(in[0]), a, "perm rank mismatch");
    TensorShape o{{}, in[0].dtype};
    for (auto d : p) o.dims.push_back(in[0].dims.at(normalize_dim(static_cast<int>(d), nd(in[0]))));
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    auto const& p = a.ints("perm");
    for (size_t i = 0; i < p.size(); ++i) o.shard_dims[i] = in[0].shard_dims.at(normalize_dim(static_cast<int>(p[i]), in[0].num_dims()));
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec reverse_spec() {
  OpSpec s = unary_spec();
  s.required = {"axis"};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    require(in[0].dim(static_cast<int>(a.i("axis"))).degree == 1, a, "reverse axis must be unpartitioned");
    return PShapes{in[0]};
  };
  return s;
}

OpSpec gather_spec() {
  OpSpec s;
  s.num_inputs = 2;
  s.required = {"dim"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    require(nd(in[0]) == nd(in[1]), a, "index rank must match input rank");
    TensorShape o = in[1];
    o.dtype = in[0].dtype;
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    int dim = normalize_dim(static_cast<int>(a.i("dim")), in[0].num_dims());
    require(in[0].shard_dims[dim].degree == 1 && in[1].shard_dims[dim].degree == 1, a, "gather dim must be unpartitioned");
    for (int d = 0; d < in[0].num_dims(); ++d)
      require(in[0].shard_dims[d].degree == in[1].shard_dims[d].degree, a, "degree mismatch");
    auto o = in[1];
    o.dtype = in[0].dtype;
    o.sum_degree = in[0].sum_degree;
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec reduce_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"axes"};
  s.defaults = {{"keepdims", false}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto axes = norm_axes(a, "axes", nd(in[0]));
    TensorShape o{{}, in[0].dtype};
    for (int d = 0; d < nd(in[0]); ++d) {
      bool red = std::find(axes.begin(), axes.end(), d) != axes.end();
      if (!red) o.dims.push_back(in[0].dims[d]);
      else if (a.b("keepdims")) o.dims.push_back(1);
    }
    if (a.type == OpType::REDUCE_ARGMAX || a.type == OpType::REDUCE_ARGMIN) o.dtype = DataType::INT64;
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto const& x = in[0];
    auto axes = norm_axes(a, "axes", x.num_dims());
    bool linear = a.type == OpType::REDUCE_SUM || a.type == OpType::REDUCE_MEAN || a.type == OpType::MEAN;
    if (!linear) require(x.sum_degree == 1, a, "nonlinear reduction of partial sums");
    auto o = registry()[static_cast<int>(a.type)].out(a, {x.reduced_shape()})[0];
    std::vector<int> deg;
    int sum = x.sum_degree;
    for (int d = 0; d < x.num_dims(); ++d) {
      bool red = std::find(axes.begin(), axes.end(), d) != axes.end();
      if (red) {
        if (x.shard_dims[d].degree > 1) {
          require(linear, a, "reducing a partitioned axis needs a linear reduction");
          sum *= x.shard_dims[d].degree;
        }
        if (a.b("keepdims")) deg.push_back(1);
      } else {
        deg.push_back(x.shard_dims[d].degree);
      }
    }
    return PShapes{lift_to_parallel_with_degrees(o, sum, x.discard_copy_degree, deg)};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec cast_spec() {
  OpSpec s = unary_spec();
  s.required = {"dtype"};
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto o = in[0];
    o.dtype = datatype_from_string(a.s("dtype"));
    return Shapes{o};
  };
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    o.dtype = datatype_from_string(a.s("dtype"));
    return PShapes{o};
  };
  return s;
}

OpSpec dropout_spec() {
  OpSpec s = unary_spec();
  s.defaults = {{"rate", 0.5}, {"seed", int64_t(0)}};
  return s;
}

OpSpec topk_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"k"};
  s.defaults = {{"sorted", true}};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto v = in[0];
    v.at(-1) = a.i("k");
    auto idx = v;
    idx.dtype = DataType::INT32;
    return Shapes{v, idx};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    require(in[0].dim(-1).degree == 1 && in[0].sum_degree == 1, a, "topk dim must be unpartitioned");
    auto v = in[0];
    v.dim(-1).size = a.i("k");
    auto idx = v;
    idx.dtype = DataType::INT32;
    return PShapes{v, idx};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec broadcast_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"target_dims"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    TensorShape o{a.ints("target_dims"), in[0].dtype};
    auto b = broadcast_dims(a, in[0].dims, o.dims);
    require(b == o.dims, a, "cannot broadcast to target");
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = registry()[static_cast<int>(OpType::BROADCAST)].out(a, {in[0].reduced_shape()})[0];
    auto p = lift_to_parallel(o);
    int off = o.num_dims() - in[0].num_dims();
    for (int d = 0; d < in[0].num_dims(); ++d) {
      if (in[0].shard_dims[d].size == o.dims[d + off]) p.shard_dims[d + off].degree = in[0].shard_dims[d].degree;
      else require(in[0].shard_dims[d].degree == 1, a, "broadcast dim must be unpartitioned");
    }
    p.sum_degree = in[0].sum_degree;
    p.discard_copy_degree = in[0].discard_copy_degree;
    return PShapes{p};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec unsqueeze_spec(bool squeeze) {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"dims"};
  s.weights = no_weights;
  s.out = [squeeze](const OpAttrs& a, const Shapes& in) {
    auto o = in[0];
    if (squeeze) {
      auto ax = norm_axes(a, "dims", nd(o));
      for (auto it = ax.rbegin(); it != ax.rend(); ++it) {
        require(o.dims[*it] == 1, a, "squeezed dim must have size 1");
        o.dims.erase(o.dims.begin() + *it);
      }
    } else {
      std::vector<int64_t> ds = a.ints("dims");
      std::sort(ds.begin(), ds.end());
      for (auto d : ds) {
        int p = static_cast<int>(d < 0 ? d + nd(o) + 1 : d);
        o.dims.insert(o.dims.begin() + p, 1);
      }
    }
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [squeeze](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    if (squeeze) {
      auto ax = norm_axes(a, "dims", o.num_dims());
      for (auto it = ax.rbegin(); it != ax.rend(); ++it) o.shard_dims.erase(o.shard_dims.begin() + *it);
    } else {
      std::vector<int64_t> ds = a.ints("dims");
      std::sort(ds.begin(), ds.end());
      for (auto d : ds) {
        int p = static_cast<int>(d < 0 ? d + o.num_dims() + 1 : d);
        o.shard_dims.insert(o.shard_dims.begin() + p, ShardParallelDim{1, 1});
      }
    }
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec slice_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"axes", "starts", "ends"};
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto o = in[0];
    auto const &ax = a.ints("axes"), &st = a.ints("starts"), &en = a.ints("ends");
    require(ax.size() == st.size() && st.size() == en.size(), a, "axes/starts/ends length mismatch");
    for (size_t i = 0; i < ax.size(); ++i) {
      int d = normalize_dim(static_cast<int>(ax[i]), nd(o));
      int64_t lo = st[i] < 0 ? st[i] + in[0].dims[d] : st[i];
      int64_t hi = en[i] < 0 ? en[i] + in[0].dims[d] : std::min(en[i], in[0].dims[d]);
      o.dims[d] = std::max<int64_t>(0, hi - lo);
    }
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    auto serial = registry()[static_cast<int>(OpType::SLICE)].out(a, {in[0].reduced_shape()})[0];
    for (auto d : a.ints("axes")) {
      int dd = normalize_dim(static_cast<int>(d), o.num_dims());
      require(o.shard_dims[dd].degree == 1, a, "sliced axis must be unpartitioned");
      o.shard_dims[dd].size = serial.dims[dd];
    }
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

OpSpec pad_spec() {
  OpSpec s;
  s.num_inputs = 1;
  s.required = {"pads"};  // [before_0, after_0, before_1, after_1, ...]
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes& in) {
    auto o = in[0];
    auto const& p = a.ints("pads");
    require(static_cast<int>(p.size()) == 2 * nd(o), a, "pads must have 2*rank entries");
    for (int d = 0; d < nd(o); ++d) o.dims[d] += p[2 * d] + p[2 * d + 1];
    return Shapes{o};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    auto const& p = a.ints("pads");
    for (int d = 0; d < o.num_dims(); ++d) {
      if (p[2 * d] || p[2 * d + 1]) {
        require(o.shard_dims[d].degree == 1, a, "padded axis must be unpartitioned");
        o.shard_dims[d].size += p[2 * d] + p[2 * d + 1];
      }
    }
    return PShapes{o};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

// ---- sources -----------------------------------------------------------------
OpSpec source_spec(OpType t) {
  OpSpec s;
  s.num_inputs = 0;
  s.required = {"dims"};
  s.defaults = {{"data_type", std::string("float")}};
  if (t == OpType::WEIGHT) s.defaults["initializer"] = std::string("{\"type\":\"zero\"}");
  s.weights = no_weights;
  s.out = [](const OpAttrs& a, const Shapes&) {
    return Shapes{TensorShape{a.ints("dims"), datatype_from_string(a.s("data_type"))}};
  };
  s.wts = no_weight_shapes;
  s.pout = [](const OpAttrs& a, const PShapes&) {
    return PShapes{lift_to_parallel(TensorShape{a.ints("dims"), datatype_from_string(a.s("data_type"))})};
  };
  s.pwts = no_pweight_shapes;
  return s;
}

// ---- parallel ops ----------------------------------------------------------
OpSpec repartition_spec() {
  OpSpec s = unary_spec();
  s.required = {"dim", "degree"};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    auto& d = o.dim(static_cast<int>(a.i("dim")));
    d.degree *= static_cast<int>(a.i("degree"));
    require(d.size % d.degree == 0, a, "dim size not divisible by new degree");
    return PShapes{o};
  };
  return s;
}
OpSpec combine_spec() {
  OpSpec s = unary_spec();
  s.required = {"dim", "degree"};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    auto& d = o.dim(static_cast<int>(a.i("dim")));
    require(d.degree % a.i("degree") == 0, a, "combine degree does not divide shard degree");
    d.degree /= static_cast<int>(a.i("degree"));
    return PShapes{o};
  };
  return s;
}
// `partial=true` replicates into partial-sum replicas (only replica 0 carries
// the value, the rest are zeros): used for biases of row-parallel Linear/Conv.
OpSpec replicate_spec() {
  OpSpec s = unary_spec();
  s.required = {"degree"};
  s.defaults = {{"partial", false}};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    if (a.b("partial")) o.sum_degree *= static_cast<int>(a.i("degree"));
    else o.discard_copy_degree *= static_cast<int>(a.i("degree"));
    return PShapes{o};
  };
  return s;
}
OpSpec reduction_spec() {
  OpSpec s = unary_spec();
  s.required = {"degree"};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    require(o.sum_degree % a.i("degree") == 0, a, "reduction degree does not divide sum degree");
    o.sum_degree /= static_cast<int>(a.i("degree"));
    return PShapes{o};
  };
  return s;
}
// AllToAll: moves `degree` of partitioning from src_dim to dst_dim
// (Ulysses sequence<->head exchange, DLRM embedding exchange).
OpSpec alltoall_spec() {
  OpSpec s = unary_spec();
  s.required = {"src_dim", "dst_dim", "degree"};
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto o = in[0];
    int k = static_cast<int>(a.i("degree"));
    auto& sd = o.dim(static_cast<int>(a.i("src_dim")));
    auto& dd = o.dim(static_cast<int>(a.i("dst_dim")));
    require(sd.degree % k == 0, a, "src degree not divisible");
    sd.degree /= k;
    dd.degree *= k;
    require(dd.size % dd.degree == 0, a, "dst dim not divisible");
    return PShapes{o};
  };
  return s;
}
OpSpec fused_parallel_spec() {
  OpSpec s = unary_spec();
  s.required = {"ops"};  // JSON array of parallel OpAttrs
  s.pout = [](const OpAttrs& a, const PShapes& in) {
    auto cur = in;
    const Json ops_j = Json::parse(a.s("ops"));
    for (auto const& j : ops_j.as_array()) {
      OpAttrs sub = normalize_attrs(OpAttrs::from_json(j));
      cur = infer_parallel_output_shapes(sub, cur);
    }
    return cur;
  };
  return s;
}

// Mixture-of-experts FFN block (the reference's MoE example builds it from
// top-k + group_by + dense experts + aggregate, examples/cpp/
// mixture_of_experts/moe.cc:159-164, with operators its vocabulary lacks).
// Inputs: x [B, D], expert ids [B, k] (int), gate weights [B, k].
// Weights: w1 [E, D, H], b1 [E, H], w2 [E, H, O], b2 [E, O].
// out[b] = sum_j gate[b, j] * expert_{id[b, j]}(x[b]).
// Expert parallelism, two lowerings:
//  * "replicated": token inputs carry discard_copy c; experts are sharded c
//    ways; each rank applies only its experts -> output sum_degree c
//    (resolved by a Reduction);
//  * "alltoall": token inputs are batch-sharded; experts are sharded
//    `expert_degree` ways across consecutive batch shards and tokens are
//    dispatched / combined with all-to-alls inside the op.
OpSpec experts_spec() {
  OpSpec s;
  s.num_inputs = 3;
  s.required = {"num_experts", "hidden_size", "out_dim"};
  s.defaults = {{"activation", std::string("relu")}, {"use_bias", true}, {"expert_degree", int64_t(1)},
                {"expert_parallel_mode", std::string("replicated")}};
  s.weights = [](const OpAttrs& a) {
    if (a.b("use_bias")) return std::vector<std::string>{"w1", "b1", "w2", "b2"};
    return std::vector<std::string>{"w1", "w2"};
  };
  s.out = [](const OpAttrs& a, const Shapes& in) {
    require(nd(in[0]) == 2, a, "x must be [batch, features]");
    require(nd(in[1]) == 2 && nd(in[2]) == 2, a, "expert ids / gates must be [batch, k]");
    require(in[1].dims == in[2].dims && in[1].dims[0] == in[0].dims[0], a, "ids / gates / x batch mismatch");
    require(in[1].dims[1] <= a.i("num_experts"), a, "k exceeds the number of experts");
    return Shapes{TensorShape{{in[0].dims[0], a.i("out_dim")}, in[0].dtype}};
  };
  s.wts = [](const OpAttrs& a, const Shapes& in) {
    const int64_t E = a.i("num_experts"), D = in[0].dims[1], H = a.i("hidden_size"), O = a.i("out_dim");
    Shapes w{TensorShape{{E, D, H}, in[0].dtype}};
    if (a.b("use_bias")) w.push_back(TensorShape{{E, H}, in[0].dtype});
    w.push_back(TensorShape{{E, H, O}, in[0].dtype});
    if (a.b("use_bias")) w.push_back(TensorShape{{E, O}, in[0].dtype});
    return w;
  };
  auto parse = [](const OpAttrs& a, const PShapes& in) {
    for (auto const& t : in) {
      require(t.num_dims() == 2, a, "rank-2 inputs");
      require(t.sum_degree == 1, a, "inputs cannot be partial sums");
      require(t.dim(1).degree == 1, a, "feature / k dims must be unpartitioned");
      require(t.dim(0).degree == in[0].dim(0).degree, a, "batch degrees differ");
      require(t.discard_copy_degree == in[0].discard_copy_degree, a, "replica degrees differ");
    }
    const int c = in[0].discard_copy_degree;
    require(a.i("num_experts") % c == 0, a, "experts not divisible by the expert degree");
    if (a.s("expert_parallel_mode") == "alltoall") {
      const int ed = static_cast<int>(a.i("expert_degree"));
      require(c == 1, a, "all-to-all expert parallelism takes batch-sharded (not replicated) tokens");
      require(ed >= 1 && in[0].dim(0).degree % ed == 0, a, "expert degree must divide the batch degree");
      require(a.i("num_experts") % ed == 0, a, "experts not divisible by the expert degree");
    }
  };
  s.pout = [parse](const OpAttrs& a, const PShapes& in) {
    parse(a, in);
    auto o = registry()[static_cast<int>(OpType::EXPERTS)].out(
        a, {in[0].reduced_shape(), in[1].reduced_shape(), in[2].reduced_shape()})[0];
    return PShapes{lift_to_parallel_with_degrees(o, in[0].discard_copy_degree, 1, {in[0].dim(0).degree, 1})};
  };
  s.pwts = [parse](const OpAttrs& a, const PShapes& in) {
    parse(a, in);
    auto ws = registry()[static_cast<int>(OpType::EXPERTS)].wts(
        a, {in[0].reduced_shape(), in[1].reduced_shape(), in[2].reduced_shape()});
    const int bx = in[0].dim(0).degree;
    int ed = in[0].discard_copy_degree, copies = bx;
    if (a.s("expert_parallel_mode") == "alltoall") {
      ed = static_cast<int>(a.i("expert_degree"));
      copies = bx / ed;
    }
    PShapes r;
    for (auto const& w : ws) {
      std::vector<int> deg(w.num_dims(), 1);
      deg[0] = ed;
      r.push_back(lift_to_parallel_with_degrees(w, 1, copies, deg));
    }
    return r;
  };
  return s;
}

OpSpec noop_spec() { return unary_spec(); }

std::unordered_map<int, OpSpec> build_registry() {
  std::unordered_map<int, OpSpec> r;
  auto put = [&](OpType t, OpSpec s) { r[static_cast<int>(t)] = std::move(s); };
  for (OpType t : all_op_types())
    if (is_elementwise_unary(t)) put(t, unary_spec());
  r[static_cast<int>(OpType::SCALAR_MULTIPLY)].required = {"scalar"};
  r[static_cast<int>(OpType::SCALAR_ADD)].required = {"scalar"};
  r[static_cast<int>(OpType::SCALAR_SUB)].required = {"scalar"};
  r[static_cast<int>(OpType::SCALAR_TRUE_DIV)].required = {"scalar"};
  r[static_cast<int>(OpType::SCALAR_FLOOR_DIV)].required = {"scalar"};
  r[static_cast<int>(OpType::POW)].required = {"exponent"};
  r[static_cast<int>(OpType::ELU)].defaults = {{"alpha", 1.0}};
  r[static_cast<int>(OpType::LEAKYRELU)].defaults = {{"alpha", 0.01}};
  r[static_cast<int>(OpType::GELU)].defaults = {{"approximate", std::string("tanh")}};
  for (OpType t : all_op_types())
    if (is_elementwise_binary(t)) put(t, binary_spec());
  put(OpType::NOOP, noop_spec());
  put(OpType::INPUT, source_spec(OpType::INPUT));
  put(OpType::WEIGHT, source_spec(OpType::WEIGHT));
  put(OpType::LINEAR, linear_spec());
  put(OpType::CONV2D, conv2d_spec());
  put(OpType::POOL2D, pool2d_spec());
  put(OpType::BATCHNORM, batchnorm_spec());
  put(OpType::LAYERNORM, layernorm_spec());
  put(OpType::SOFTMAX, softmax_spec());
  put(OpType::EMBEDDING, embedding_spec());
  put(OpType::MULTIHEAD_ATTENTION, mha_spec());
  put(OpType::BATCHMATMUL, batch_matmul_spec());
  put(OpType::MATMUL, batch_matmul_spec());
  put(OpType::CONCAT, concat_spec());
  put(OpType::SPLIT, split_spec());
  put(OpType::FLAT, flat_spec());
  put(OpType::RESHAPE, reshape_spec());
  put(OpType::TRANSPOSE, transpose_spec());
  put(OpType::REVERSE, reverse_spec());
  put(OpType::GATHER, gather_spec());
  for (OpType t : {OpType::REDUCE_SUM, OpType::REDUCE_MEAN, OpType::REDUCE_MAX, OpType::REDUCE_MIN,
                   OpType::REDUCE_PROD, OpType::REDUCE_ARGMAX, OpType::REDUCE_ARGMIN, OpType::MEAN})
    put(t, reduce_spec());
  put(OpType::CAST, cast_spec());
  put(OpType::DROPOUT, dropout_spec());
  put(OpType::TOPK, topk_spec());
  put(OpType::BROADCAST, broadcast_spec());
  put(OpType::UNSQUEEZE, unsqueeze_spec(false));
  put(OpType::SQUEEZE, unsqueeze_spec(true));
  put(OpType::SLICE, slice_spec());
  put(OpType::PAD, pad_spec());
  put(OpType::REPARTITION, repartition_spec());
  put(OpType::COMBINE, combine_spec());
  put(OpType::REPLICATE, replicate_spec());
  put(OpType::REDUCTION, reduction_spec());
  put(OpType::ALLTOALL, alltoall_spec());
  put(OpType::FUSED_PARALLEL, fused_parallel_spec());
  put(OpType::EXPERTS, experts_spec());
  return r;
}

std::unordered_map<int, OpSpec>& registry() {
  static std::unordered_map<int, OpSpec> r = build_registry();
  return r;
}

const OpSpec& spec_of(const OpAttrs& a) {
  auto& r = registry();
  auto it = r.find(static_cast<int>(a.type));
  if (it == r.end()) throw FFError("operator " + to_string(a.type) + " has no shape rules");
  return it->second;
}

}  // namespace

// ---------------------------------------------------------------------------
OpAttrs normalize_attrs(OpAttrs attrs) {
  auto const& sp = spec_of(attrs);
  for (auto const& k : sp.required)
    if (!attrs.has(k)) throw FFError(to_string(attrs.type) + ": missing required attribute '" + k + "'");
  for (auto const& kv : sp.defaults)
    if (!attrs.has(kv.first)) attrs.attrs[kv.first] = kv.second;
  return attrs;
}

int num_weights(const OpAttrs& a) { return static_cast<int>(spec_of(a).weights(a).size()); }
int num_data_inputs(const OpAttrs& a) { return spec_of(a).num_inputs; }
std::vector<std::string> weight_names(const OpAttrs& a) { return spec_of(a).weights(a); }

static void check_arity(const OpAttrs& a, size_t n) {
  int k = spec_of(a).num_inputs;
  if (k >= 0 && static_cast<size_t>(k) != n)
    throw FFError(to_string(a.type) + ": expected " + std::to_string(k) + " inputs, got " + std::to_string(n));
}

std::vector<TensorShape> infer_output_shapes(const OpAttrs& a, const std::vector<TensorShape>& inputs) {
  check_arity(a, inputs.size());
  return spec_of(a).out(a, inputs);
}
std::vector<TensorShape> infer_weight_shapes(const OpAttrs& a, const std::vector<TensorShape>& inputs) {
  check_arity(a, inputs.size());
  return spec_of(a).wts(a, inputs);
}
std::vector<ParallelTensorShape> infer_parallel_output_shapes(const OpAttrs& a,
                                                              const std::vector<ParallelTensorShape>& inputs) {
  check_arity(a, inputs.size());
  for (auto const& x : inputs)
    if (!x.is_valid()) throw FFError(to_string(a.type) + ": invalid input parallel shape " + x.str());
  auto r = spec_of(a).pout(a, inputs);
  for (auto const& x : r)
    if (!x.is_valid()) throw FFError(to_string(a.type) + ": produces invalid parallel shape " + x.str());
  return r;
}
std::vector<ParallelTensorShape> infer_parallel_weight_shapes(const OpAttrs& a,
                                                              const std::vector<ParallelTensorShape>& inputs) {
  check_arity(a, inputs.size());
  auto r = spec_of(a).pwts(a, inputs);
  for (auto const& x : r)
    if (!x.is_valid()) throw FFError(to_string(a.type) + ": invalid weight parallel shape " + x.str());
  return r;
}
bool is_valid_parallelization(const OpAttrs& a, const std::vector<ParallelTensorShape>& inputs) {
  try {
    infer_parallel_output_shapes(a, inputs);
    infer_parallel_weight_shapes(a, inputs);
    return true;
  } catch (FFError const&) {
    return false;
  }
}

// ---------------------------------------------------------------------------
OpWork estimate_op_work(const OpAttrs& a, const std::vector<TensorShape>& in,
                        const std::vector<TensorShape>& w, const std::vector<TensorShape>& out) {
  OpWork r;
  double bytes = 0;
  for (auto const& t : in) bytes += static_cast<double>(t.size_bytes());
  for (auto const& t : w) bytes += static_cast<double>(t.size_bytes());
  for (auto const& t : out) bytes += static_cast<double>(t.size_bytes());
  r.bytes = bytes;
  auto n_out = out.empty() ? 0.0 : static_cast<double>(out[0].num_elements());
  switch (a.type) {
    case OpType::LINEAR: {
      double m = static_cast<double>(in[0].num_elements() / in[0].at(-1));
      double k = static_cast<double>(in[0].at(-1));
      double n = static_cast<double>(out[0].at(-1));
      r.flops = 2 * m * k * n;
      r.matmul_like = true;
      double mn = std::min({m, n, k});
      r.mfma_efficiency_hint = std::min(1.0, mn / 256.0 + 0.15);
      break;
    }
    case OpType::CONV2D: {
      double kk = static_cast<double>(w[0].num_elements() / w[0].dims[0]);
      r.flops = 2 * n_out * kk;
      r.matmul_like = true;
      r.mfma_efficiency_hint = std::min(1.0, static_cast<double>(out[0].dims[1]) / 256.0 + 0.25);
      break;
    }
    case OpType::BATCHMATMUL:
    case OpType::MATMUL: {
      double k = static_cast<double>(in[0].at(-1));
      r.flops = 2 * n_out * k;
      r.matmul_like = true;
      r.mfma_efficiency_hint = std::min(1.0, k / 256.0 + 0.2);
      break;
    }
    case OpType::MULTIHEAD_ATTENTION: {
      double b = static_cast<double>(in[0].dims[0]);
      double sq = static_cast<double>(in[0].dims[1]);
      double sk = static_cast<double>(in[1].dims[1]);
      double h = static_cast<double>(w[0].dims[1]);  // local heads
      double p = static_cast<double>(w[0].dims[0]);
      double kd = a.i("kdim") > 0 ? static_cast<double>(a.i("kdim")) : static_cast<double>(a.i("embed_dim")) / static_cast<double>(a.i("num_heads"));
      // projections: every token through its per-head parameter block
      r.flops = 2 * b * sq * p * h + 4 * b * h * sq * sk * kd;
      if (a.b("causal")) r.flops -= 2 * b * h * sq * sk * kd;
      r.matmul_like = true;
      r.mfma_efficiency_hint = 0.8;
      break;
    }
    case OpType::EXPERTS: {
      // dropless routing: B*k token-expert pairs through two GEMMs, spread
      // evenly over the expert shards of this piece
      const double pairs = static_cast<double>(in[1].dims[0]) * static_cast<double>(in[1].dims[1]);
      const double E = static_cast<double>(a.i("num_experts")), El = static_cast<double>(w[0].dims[0]);
      const double D = static_cast<double>(in[0].dims[1]), H = static_cast<double>(a.i("hidden_size"));
      const double O = static_cast<double>(a.i("out_dim"));
      r.flops = 2 * pairs * (El / E) * (D * H + H * O);
      r.bytes = static_cast<double>(w[0].size_bytes()) * (1 + (O / D)) + 4 * pairs * (D + O);
      r.matmul_like = true;
      r.mfma_efficiency_hint = std::min(1.0, pairs * (El / E) / El / 512.0 + 0.2);
      break;
    }
    case OpType::EMBEDDING:
      r.flops = n_out;
      // only the gathered rows are read, not the whole table
      r.bytes = static_cast<double>(in[0].size_bytes()) + 2 * static_cast<double>(out[0].size_bytes());
      break;
    case OpType::LAYERNORM:
    case OpType::BATCHNORM:
    case OpType::SOFTMAX:
      r.flops = 8 * n_out;
      break;
    case OpType::POOL2D:
      r.flops = n_out * static_cast<double>(a.i("kernel_h") * a.i("kernel_w"));
      break;
    case OpType::INPUT:
    case OpType::WEIGHT:
    case OpType::NOOP:
    case OpType::REPARTITION:
    case OpType::COMBINE:
    case OpType::REPLICATE:
    case OpType::REDUCTION:
    case OpType::ALLTOALL:
    case OpType::FUSED_PARALLEL:
    case OpType::RESHAPE:
    case OpType::FLAT:
    case OpType::UNSQUEEZE:
    case OpType::SQUEEZE:
      r.flops = 0;
      r.bytes = 0;
      break;
    default:
      r.flops = n_out;
  }
  return r;
}

OpAttrs make_linear(int64_t out_channels, bool use_bias, Activation act) {
  OpAttrs a(OpType::LINEAR);
  a.set("out_channels", out_channels).set("use_bias", use_bias).set("activation", to_string(act));
  return normalize_attrs(a);
}
OpAttrs make_repartition(int dim, int degree) {
  return normalize_attrs(OpAttrs(OpType::REPARTITION).set("dim", dim).set("degree", degree));
}
OpAttrs make_combine(int dim, int degree) {
  return normalize_attrs(OpAttrs(OpType::COMBINE).set("dim", dim).set("degree", degree));
}
OpAttrs make_replicate(int degree) { return normalize_attrs(OpAttrs(OpType::REPLICATE).set("degree", degree)); }
OpAttrs make_reduction(int degree) { return normalize_attrs(OpAttrs(OpType::REDUCTION).set("degree", degree)); }

}  // namespace ff
