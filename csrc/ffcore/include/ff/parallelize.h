// Per-layer parallelization configs and their lowering to a PCG.
//
// Parity: the legacy MCMC search (lib/runtime/src/model.cc
// strategy_search_task / Simulator::simulate_runtime, §3.5) searched over a
// ParallelConfig {device_type, nDims, dim[], device_ids[]} per op; the new
// stack expresses the same choices as parallel ops in a PCG (§2.7:
// Linear column/row parallel linear.cc:86-136, attention head parallel
// attention.cc:241-352, embedding out-channel embedding.cc:88-112).
//
// Here a LayerConfig = {batch degree, sequence degree, model degree, kind};
// `lower_strategy` turns a CG + {layer -> config} into a PCG by converting
// every data edge to the consumer's required parallel shape with the
// minimal Reduction / Combine / Repartition / Replicate chain (weights get
// the degrees their consumer's shape rules require).
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/json.h"

namespace ff {

enum class MPKind { NONE = 0, COLUMN = 1, ROW = 2, HEADS = 3, EXPERTS = 4 };
std::string mp_kind_to_string(MPKind k);
MPKind mp_kind_from_string(const std::string& s);

struct LayerConfig {
  int batch = 1;   // degree on dim 0 (sample)
  int seq = 1;     // degree on dim 1 of rank>=3 activations (attribute / sequence parallel)
  int model = 1;   // degree of the model-parallel split
  MPKind kind = MPKind::NONE;
  int total() const { return batch * seq * model; }
  bool operator==(const LayerConfig& o) const {
    return batch == o.batch && seq == o.seq && model == o.model && kind == o.kind;
  }
  bool operator!=(const LayerConfig& o) const { return !(*this == o); }
  bool operator<(const LayerConfig& o) const;
  std::string str() const;
  Json to_json() const;
  static LayerConfig from_json(const Json& j);
};

using StrategyConfig = std::map<int, LayerConfig>;  // CG node id -> config

struct SearchSpaceOptions {
  bool enable_parameter_parallel = true;   // model-parallel kinds (COLUMN/ROW/HEADS)
  bool enable_attribute_parallel = false;  // sequence-dim degrees
  bool allow_partial_world = false;        // configs whose total degree < world (implicit replicas)
  int max_model_degree = 8;
};

// Candidate configs for one CG layer on `world` devices (total degree == world
// unless allow_partial_world).  Always contains the data-parallel config (or
// the replicated one when the batch does not divide).
std::vector<LayerConfig> candidate_configs(const ComputationGraph& cg, int node, int world,
                                           const SearchSpaceOptions& opt = {});
StrategyConfig data_parallel_strategy(const ComputationGraph& cg, int world);

// Required data-input parallel shapes of `node` under `cfg` (nullopt if the op
// cannot be parallelized that way).
std::optional<std::vector<ParallelTensorShape>> required_input_shapes(const ComputationGraph& cg, int node,
                                                                      const LayerConfig& cfg);
// The layer's attrs as lowered under `cfg` (all-to-all expert parallelism
// records its expert degree on the op).
OpAttrs configured_op(const OpAttrs& op, const LayerConfig& cfg);

struct Lowering {
  ParallelComputationGraph pcg;
  std::map<int, int> cg_to_pcg;  // CG layer -> PCG layer
  int num_parallel_ops = 0;
};
// Throws FFError if a config is inconsistent with the graph.
Lowering lower_strategy(const ComputationGraph& cg, const StrategyConfig& cfg, int world);

// Insert the minimal parallel-op chain converting `v` to `target` (same
// logical shape).  Exposed for tests and substitutions.
ValueRef convert_parallel_shape(ParallelComputationGraph& pcg, ValueRef v, const ParallelTensorShape& target,
                                int* num_ops = nullptr);

Json strategy_to_json(const ComputationGraph& cg, const StrategyConfig& s);
StrategyConfig strategy_from_json(const ComputationGraph& cg, const Json& j);

}  // namespace ff
