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
  enum Kind { EQUAL = 0, DIVISIBLE_BY = 1 } kind = EQUAL;
  std::string key;
  AttrValue value;
};

struct OperatorPattern {
  std::optional<OpType> type;
  std::vector<AttrConstraint> attrs;
  int num_data_inputs = -1;  // -1: any
  bool satisfied_by(const OpAttrs& op) const;
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
};

std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  size_t max_matches = 1u << 20);
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
// Converts rules whose weight handling is expressible with implicit weights
// (weights never rewritten); nullopt otherwise.
std::optional<Substitution> substitution_from_legacy_rule(const LegacyRule& r);

}  // namespace ff
