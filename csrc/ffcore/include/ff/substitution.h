// Graph substitutions over the PCG: patterns, matching, output graphs,
// application, the built-in parallelization rule set and the legacy TASO
// rule corpus.
//
// Parity:
//  * PCGPattern / OperatorAttributePattern / TensorAttributePattern:
//    lib/substitutions/include/substitutions/pcg_pattern.struct.toml,
//    operator_pattern/*, tensor_pattern/* (constraints over attribute keys)
//  * find_pattern_matches: substitutions/unlabelled/find_pattern_matches.cc:17-115
//  * OutputGraphExpr + apply_substitution: substitution.cc:25-167,
//    output_graph/materialize_operator_from_attrs_map.cc,
//    substitution_internal/perform_shape_inference.cc
//  * legacy rule corpus loader: lib/substitution-generator/src/.../legacy_rules.cc:10-66
//    (substitutions/graph_subst_3_v2.json, 640 rules)
//  * rule -> dot: bin/substitution-to-dot/substitution_to_dot.cc:17-152
//
// Differences by design: patterns are over DATA edges only — an operator's
// weights are not pattern inputs but are re-created by `apply_substitution`
// with the parallel shape the rewritten operator requires (the PCG's weight
// chain = WEIGHT + parallel ops, generate_weight_transform).  Matching is a
// connected backtracking search anchored on the rarest pattern operator.
#pragma once
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/json.h"

namespace ff {

struct PatternValue {
  int node = -1;  // >= 0: pattern/output node; < 0: pattern input (-node - 1)
  int idx = 0;
  static PatternValue input(int k) { return {-k - 1, 0}; }
  bool is_input() const { return node < 0; }
  int input_index() const { return -node - 1; }
  bool operator==(const PatternValue& o) const { return node == o.node && idx == o.idx; }
};

struct AttrConstraint {
  // DIM_FROM_END: an axis attribute counted from the last dimension of the
  // operator's first data input (value -1 = last dim), compared after
  // normalising the attribute against that input's rank -- the legacy TASO
  // rules number dims innermost-first and never state the rank
  enum Kind { EQUAL = 0, DIVISIBLE_BY = 1, DIM_FROM_END = 2 } kind = EQUAL;
  std::string key;
  AttrValue value;
};

struct OperatorPattern {
  std::optional<OpType> type;
  std::vector<AttrConstraint> attrs;
  int num_data_inputs = -1;  // -1: any
  int num_outputs = -1;      // -1: any
  // rank: of the operator's first data input (-1 unknown: DIM_FROM_END fails)
  bool satisfied_by(const OpAttrs& op, int rank = -1) const;
};

struct PCGPattern {
  std::vector<OperatorPattern> nodes;
  std::vector<std::vector<PatternValue>> inputs;  // per node: data inputs
  int num_inputs = 0;
  std::vector<PatternValue> outputs;               // exposed outputs
  int add_node(OperatorPattern p, std::vector<PatternValue> ins);
};

struct PCGPatternMatch {
  std::vector<int> node_map;         // pattern node -> PCG node
  std::vector<ValueRef> input_map;   // pattern input -> PCG value
};

struct AttrAssignment {
  std::string key;
  bool copy = false;         // copy from a matched pattern node
  int from_node = -1;
  std::string from_key;
  AttrValue value;           // constant
};

struct OutputOperator {
  int copy_from = -1;        // >= 0: start from the matched pattern node's attrs
  OpType type = OpType::NOOP;
  std::vector<AttrAssignment> assign;
  std::vector<PatternValue> inputs;  // node < 0: pattern input; else output node
  std::string name;          // optional; else derived from copy_from
};

struct Substitution {
  std::string name;
  PCGPattern pattern;
  std::vector<OutputOperator> out_nodes;
  std::vector<PatternValue> output_mapping;  // per pattern output: output value (node<0: pattern input)
  Json to_json() const;
  static Substitution from_json(const Json& j);  // inverse of to_json
};

// A rule set file: either the legacy TASO corpus ({"rule": [...]}, every
// convertible rule) or a list of Substitution::to_json() objects
// ({"substitutions": [...]}); `skipped` receives the legacy rules that could
// not be converted (name + reason).
std::vector<Substitution> load_substitutions(const Json& j, std::vector<std::string>* skipped = nullptr);
std::vector<Substitution> load_substitutions_file(const std::string& path, std::vector<std::string>* skipped = nullptr);

// Per-PCG lookup tables every pattern match reads (data nodes by operator
// type, data inputs, input rank, value users): built once per PCG, shared
// by all the rules tried on it (the Unity search tries every rule on every
// popped state).
struct PatternMatchIndex {
  explicit PatternMatchIndex(const ParallelComputationGraph& pcg);
  std::vector<int> data_nodes;                             // topological order
  std::map<OpType, std::vector<int>> by_type;
  std::vector<char> weight_path;                           // by node id
  std::vector<int> rank;                                   // rank of the first data input (-1 none)
  std::vector<std::vector<ValueRef>> din;                  // data inputs by node id
  std::vector<std::vector<std::vector<std::pair<int, int>>>> users;  // [node][output] -> (user, slot)
  const std::vector<std::pair<int, int>>& users_of(const ValueRef& v) const;
};

std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  size_t max_matches = 1u << 20);
std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  const PatternMatchIndex& ix, size_t max_matches = 1u << 20);
// nullopt if the rewritten graph fails shape inference.
std::optional<ParallelComputationGraph> apply_substitution(const ParallelComputationGraph& pcg,
                                                           const Substitution& s, const PCGPatternMatch& m);
// Removes weight-path / parallel nodes whose outputs are unused.
void remove_dead_parallel_nodes(ParallelComputationGraph& pcg);

// Built-in parallelization rules for the degrees dividing `world`:
// partition-on-sample around every compute op type present, Linear
// column/row, attention heads, embedding channels, Combine∘Repartition and
// Repartition∘Combine cancellation, Reduction∘Replicate → all-reduce-in-place.
std::vector<Substitution> generate_parallelization_substitutions(const ParallelComputationGraph& pcg, int world);

// ---------------------------------------------------------------------------
// Legacy TASO rule corpus
struct LegacyTensor {
  int op_id = 0;
  int ts_id = 0;
};
struct LegacyOperator {
  std::string type;
  std::vector<LegacyTensor> inputs;
  std::vector<std::pair<std::string, int>> params;
  int param(const std::string& k, int dflt = -1) const;
};
struct LegacyMapOutput {
  int src_op = 0, src_ts = 0, dst_op = 0, dst_ts = 0;
};
struct LegacyRule {
  std::string name;
  std::vector<LegacyOperator> src, dst;
  std::vector<LegacyMapOutput> mapped_outputs;
};
struct LegacyRuleCollection {
  std::vector<LegacyRule> rules;
};
LegacyRuleCollection load_legacy_rules(const Json& j);
std::string legacy_rule_to_dot(const LegacyRule& r);
// Converts a legacy rule.  Weights are implicit here (a PCG operator's
// weights take the parallel shape its data inputs imply, re-created on
// apply), so the legacy rule's weight-side parallel operators (Replicate /
// Partition / Combine chains that end in a Linear's weight slot) are implied
// by the data side and dropped.  Dims are innermost-first in the legacy
// format and become DIM_FROM_END constraints / negative axes.  nullopt (with
// `why`) for a rule that still cannot be expressed.
std::optional<Substitution> substitution_from_legacy_rule(const LegacyRule& r, std::string* why = nullptr);
// The same equivalence read right to left (dst becomes the pattern).
LegacyRule reverse_legacy_rule(const LegacyRule& r);

}  // namespace ff
