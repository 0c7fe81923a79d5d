// ComputationGraph (serial) and ParallelComputationGraph (PCG) plus builders.
//
// Parity:
//  * CG layers LayerAttrs{op attrs, name}, tensors TensorAttrs{shape,
//    initializer, create_gradients}: lib/pcg/src/pcg/computation_graph.cc:23-232
//  * builder API: lib/pcg/include/pcg/computation_graph_builder.h:10-290
//  * PCG + builder (explicit WEIGHT layers followed by the parallel ops from
//    generate_weight_transform): lib/pcg/include/pcg/parallel_computation_graph/
//    parallel_computation_graph_builder.h:10-180, .cc:588-727
//  * file format v1 (JSON): lib/pcg/include/pcg/file_format/v1/*
//  * dot export: computation_graph.cc:200-232
#pragma once
#include <optional>
#include <string>
#include <vector>

#include "ff/graph.h"
#include "ff/op_attrs.h"

namespace ff {

struct LayerAttrs {
  OpAttrs op;
  std::string name;
  bool operator==(const LayerAttrs& o) const { return op == o.op && name == o.name; }
};

struct TensorAttrs {
  TensorShape shape;
  bool create_grad = true;
  std::string initializer;  // JSON (weights only)
  bool operator==(const TensorAttrs& o) const {
    return shape == o.shape && create_grad == o.create_grad && initializer == o.initializer;
  }
};

struct ParallelTensorAttrs {
  ParallelTensorShape shape;
  bool create_grad = true;
  std::string initializer;
  bool operator==(const ParallelTensorAttrs& o) const {
    return shape == o.shape && create_grad == o.create_grad && initializer == o.initializer;
  }
};

std::string default_initializer(OpType op, const std::string& weight_name);

// ---------------------------------------------------------------------------
class ComputationGraph {
 public:
  using Graph = DataflowGraph<LayerAttrs, TensorAttrs>;
  Graph g;

  ValueRef create_input(const TensorShape& shape, bool create_grad = true, const std::string& name = "");
  // A constant input (no sample dimension): data-parallel strategies replicate
  // it instead of partitioning its first dimension.
  void set_input_replicated(int node);
  ValueRef create_weight(const TensorShape& shape, const std::string& initializer, bool create_grad = true,
                         const std::string& name = "");
  // Adds an operator layer; creates its weight layers (with the given or
  // default initializers) and returns the output tensors.
  std::vector<ValueRef> add_layer(const OpAttrs& op, const std::vector<ValueRef>& inputs,
                                  const std::string& name = "",
                                  const std::vector<std::string>& weight_initializers = {});
  // Adds an operator whose weights are passed explicitly (inputs + weights).
  std::vector<ValueRef> add_layer_with_weights(const OpAttrs& op, const std::vector<ValueRef>& inputs,
                                               const std::vector<ValueRef>& weights,
                                               const std::string& name = "");

  // --- builder helpers (computation_graph_builder.h) ---
  ValueRef dense(ValueRef x, int64_t out_dim, Activation act = Activation::NONE, bool use_bias = true,
                 const std::string& name = "", const std::string& kernel_init = "",
                 const std::string& bias_init = "");
  ValueRef conv2d(ValueRef x, int64_t out_channels, int kh, int kw, int sh, int sw, int ph, int pw,
                  Activation act = Activation::NONE, int groups = 1, bool use_bias = true,
                  const std::string& name = "");
  ValueRef pool2d(ValueRef x, int kh, int kw, int sh, int sw, int ph, int pw, const std::string& pool_type,
                  Activation act = Activation::NONE, const std::string& name = "");
  ValueRef embedding(ValueRef x, int64_t num_entries, int64_t out_dim, const std::string& aggr,
                     DataType dtype = DataType::FLOAT, const std::string& name = "",
                     const std::string& kernel_init = "");
  ValueRef multihead_attention(ValueRef q, ValueRef k, ValueRef v, int64_t embed_dim, int64_t num_heads,
                               int64_t kdim = 0, int64_t vdim = 0, double dropout = 0.0,
                               bool bias = true, bool causal = false, const std::string& name = "");
  ValueRef layer_norm(ValueRef x, const std::vector<int64_t>& axes, bool affine = true, double eps = 1e-5,
                      const std::string& name = "");
  ValueRef batch_norm(ValueRef x, bool relu = true, const std::string& name = "");
  ValueRef softmax(ValueRef x, int dim = -1, const std::string& name = "");
  ValueRef unary(OpType t, ValueRef x, const std::string& name = "", std::optional<double> scalar = {});
  ValueRef binary(OpType t, ValueRef a, ValueRef b, const std::string& name = "");
  ValueRef batch_matmul(ValueRef a, ValueRef b, const std::string& name = "");
  ValueRef concat(const std::vector<ValueRef>& xs, int axis, const std::string& name = "");
  std::vector<ValueRef> split(ValueRef x, const std::vector<int64_t>& sizes, int axis,
                              const std::string& name = "");
  ValueRef flat(ValueRef x, const std::string& name = "");
  ValueRef reshape(ValueRef x, const std::vector<int64_t>& shape, const std::string& name = "");
  ValueRef transpose(ValueRef x, const std::vector<int64_t>& perm, const std::string& name = "");
  ValueRef reverse(ValueRef x, int axis, const std::string& name = "");
  ValueRef gather(ValueRef x, ValueRef index, int dim, const std::string& name = "");
  ValueRef dropout(ValueRef x, double rate, int64_t seed = 0, const std::string& name = "");
  ValueRef cast(ValueRef x, DataType dt, const std::string& name = "");
  ValueRef reduce(OpType t, ValueRef x, const std::vector<int64_t>& axes, bool keepdims,
                  const std::string& name = "");
  std::vector<ValueRef> top_k(ValueRef x, int k, bool sorted, const std::string& name = "");

  const TensorShape& shape(ValueRef v) const { return g.tensor(v).shape; }
  std::vector<int> layers_in_topo_order() const { return g.topo_order(); }
  // weights of a layer (in order) / data inputs of a layer
  std::vector<ValueRef> layer_weights(int node) const;
  std::vector<ValueRef> layer_data_inputs(int node) const;
  std::optional<int> find_layer(const std::string& name) const;

  Json to_json() const;
  static ComputationGraph from_json(const Json& j);
  std::string as_dot() const;

 private:
  std::string unique_name(const std::string& base, OpType t);
  int name_counter_ = 0;
};

// ---------------------------------------------------------------------------
class ParallelComputationGraph {
 public:
  using Graph = DataflowGraph<LayerAttrs, ParallelTensorAttrs>;
  Graph g;

  ValueRef add_input(const ParallelTensorShape& shape, bool create_grad = true, const std::string& name = "");
  // A WEIGHT layer holding `serial_shape`, followed by the parallel ops that
  // bring it to `target` (generate_weight_transform).
  ValueRef add_weight(const TensorShape& serial_shape, const ParallelTensorShape& target,
                      const std::string& initializer, bool create_grad = true, const std::string& name = "");
  // Adds an operator; inputs = data inputs followed by weights, all existing.
  std::vector<ValueRef> add_layer(const OpAttrs& op, const std::vector<ValueRef>& inputs,
                                  const std::string& name = "");
  // Adds an operator creating its weights with the degrees it requires.
  std::vector<ValueRef> add_layer_auto_weights(const OpAttrs& op, const std::vector<ValueRef>& data_inputs,
                                               const std::string& name = "",
                                               const std::vector<std::string>& weight_initializers = {});

  ValueRef parallel_partition(ValueRef x, int dim, int degree, const std::string& name = "");
  ValueRef parallel_combine(ValueRef x, int dim, int degree, const std::string& name = "");
  ValueRef parallel_replicate(ValueRef x, int degree, const std::string& name = "");
  ValueRef parallel_reduce(ValueRef x, int degree, const std::string& name = "");

  const ParallelTensorShape& shape(ValueRef v) const { return g.tensor(v).shape; }
  std::vector<ValueRef> layer_weights(int node) const;
  std::vector<ValueRef> layer_data_inputs(int node) const;
  // Operator nodes (excludes INPUT/WEIGHT and the parallel ops that feed only weights).
  bool is_weight_path(int node) const;

  // Re-run parallel shape inference over the whole graph (after a rewrite).
  void reinfer_shapes();
  Json to_json() const;
  static ParallelComputationGraph from_json(const Json& j);
  std::string as_dot() const;
  // Structural hash & equality (node ids ignored), used by Unity's state set.
  size_t structural_hash() const;
  bool structurally_equal(const ParallelComputationGraph& o) const;
  int num_operator_nodes() const;
};

std::vector<OpAttrs> generate_weight_transform(const TensorShape& serial, const ParallelTensorShape& target);

// Lift a CG to a PCG with all degrees 1.  `mapping` (if non-null) receives
// CG node id -> PCG node id.
ParallelComputationGraph pcg_from_computation_graph(const ComputationGraph& cg,
                                                    std::map<int, int>* mapping = nullptr);

// Data-parallel PCG of `cg` at `degree` (Repartition of every input's sample
// dim, weights replicated, Combine at the sinks) — the reference's
// --only-data-parallel baseline (model.h:37-39, compiler.h:11-13).
ParallelComputationGraph data_parallel_pcg(const ComputationGraph& cg, int degree);

}  // namespace ff
