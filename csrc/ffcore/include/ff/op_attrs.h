// Operator attributes + shape inference (serial and parallel).
//
// Design: every operator is `OpAttrs{type, attrs}` where `attrs` is an ordered
// key->value map.  This gives every operator value semantics, hashing, JSON
// round-trip and printing for free (the reference gets the same properties by
// code-generating ~30 typed structs, `lib/op-attrs/include/op-attrs/ops/*.struct.toml`),
// and it makes substitution attribute patterns (OperatorAttributeKey,
// `lib/substitutions/include/substitutions/operator_pattern/operator_attribute_key.enum.toml`)
// a plain key lookup.  Per-op schemas (required keys + defaults) and shape
// rules live in a registry in op_attrs.cc.
//
// Parity (semantics reproduced):
//  * serial dispatch: lib/op-attrs/src/op-attrs/get_output_shapes.cc:24-87
//  * Linear DP/TP-column/TP-row rules: lib/op-attrs/src/op-attrs/ops/linear.cc:73-140
//  * Attention batch/head rules: lib/op-attrs/src/op-attrs/ops/attention.cc:216-353
//  * Embedding out-channel (parameter) parallel: ops/embedding.cc:63-112
//  * Conv2D channel/sample parallel: ops/conv_2d.cc:24-142
//  * LayerNorm/Softmax restrictions: ops/layer_norm.cc:108-125, ops/softmax.cc:30-40
//  * Parallel ops: ops/repartition.cc, combine.cc, replicate.cc, reduction.cc
#pragma once
#include <map>
#include <string>
#include <variant>
#include <vector>

#include "ff/types.h"

namespace ff {

using AttrValue = std::variant<int64_t, double, bool, std::string, std::vector<int64_t>>;

Json attr_to_json(const AttrValue& v);
AttrValue attr_from_json(const Json& j);
std::string attr_to_string(const AttrValue& v);

struct OpAttrs {
  OpType type = OpType::NOOP;
  std::map<std::string, AttrValue> attrs;

  OpAttrs() = default;
  explicit OpAttrs(OpType t) : type(t) {}

  bool has(const std::string& k) const { return attrs.count(k) > 0; }
  int64_t i(const std::string& k) const;
  double f(const std::string& k) const;
  bool b(const std::string& k) const;
  const std::string& s(const std::string& k) const;
  const std::vector<int64_t>& ints(const std::string& k) const;

  OpAttrs& set(const std::string& k, int64_t v) { attrs[k] = v; return *this; }
  OpAttrs& set(const std::string& k, int v) { attrs[k] = static_cast<int64_t>(v); return *this; }
  OpAttrs& set(const std::string& k, double v) { attrs[k] = v; return *this; }
  OpAttrs& set(const std::string& k, bool v) { attrs[k] = v; return *this; }
  OpAttrs& set(const std::string& k, const char* v) { attrs[k] = std::string(v); return *this; }
  OpAttrs& set(const std::string& k, std::string v) { attrs[k] = std::move(v); return *this; }
  OpAttrs& set(const std::string& k, std::vector<int64_t> v) { attrs[k] = std::move(v); return *this; }

  bool operator==(const OpAttrs& o) const { return type == o.type && attrs == o.attrs; }
  bool operator!=(const OpAttrs& o) const { return !(*this == o); }
  bool operator<(const OpAttrs& o) const {
    return type != o.type ? type < o.type : attrs < o.attrs;
  }
  size_t hash() const;
  std::string str() const;
  Json to_json() const;
  static OpAttrs from_json(const Json& j);
};

// Fills defaults and validates required keys for `attrs.type`.
OpAttrs normalize_attrs(OpAttrs attrs);

// Number of weight tensors the op consumes (after its data inputs).
int num_weights(const OpAttrs& attrs);
// -1 = variadic
int num_data_inputs(const OpAttrs& attrs);
std::vector<std::string> weight_names(const OpAttrs& attrs);

// Serial shape inference.
std::vector<TensorShape> infer_output_shapes(const OpAttrs& attrs,
                                             const std::vector<TensorShape>& inputs);
std::vector<TensorShape> infer_weight_shapes(const OpAttrs& attrs,
                                             const std::vector<TensorShape>& inputs);

// Parallel shape inference.  Throws FFError if the input degrees are not a
// legal parallelisation for the op.
std::vector<ParallelTensorShape> infer_parallel_output_shapes(
    const OpAttrs& attrs, const std::vector<ParallelTensorShape>& inputs);
std::vector<ParallelTensorShape> infer_parallel_weight_shapes(
    const OpAttrs& attrs, const std::vector<ParallelTensorShape>& inputs);
// Non-throwing legality test.
bool is_valid_parallelization(const OpAttrs& attrs, const std::vector<ParallelTensorShape>& inputs);

// Per-op work estimates used by the analytic cost model (forward only;
// the cost model scales for backward).  Shapes are per-device pieces.
struct OpWork {
  double flops = 0;       // forward FLOPs
  double bytes = 0;       // forward HBM bytes moved (inputs+weights+outputs)
  bool matmul_like = false;
  double mfma_efficiency_hint = 1.0;  // small-tile penalty etc.
};
OpWork estimate_op_work(const OpAttrs& attrs, const std::vector<TensorShape>& inputs,
                        const std::vector<TensorShape>& weights,
                        const std::vector<TensorShape>& outputs);

// Convenience constructors mirroring computation_graph_builder.h
OpAttrs make_linear(int64_t out_channels, bool use_bias, Activation act = Activation::NONE);
OpAttrs make_repartition(int dim, int degree);
OpAttrs make_combine(int dim, int degree);
OpAttrs make_replicate(int degree);
OpAttrs make_reduction(int degree);

}  // namespace ff

namespace std {
template <>
struct hash<ff::OpAttrs> {
  size_t operator()(const ff::OpAttrs& a) const { return a.hash(); }
};
}  // namespace std
