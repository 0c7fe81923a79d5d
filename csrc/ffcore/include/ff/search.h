// Strategy search: MCMC over per-layer parallel configs (legacy
// strategy_search_task) and Unity best-first search over PCG substitutions
// costed by the machine-mapping DP or the simulator (graph_optimize).
//
// Parity:
//  * MCMC: lib/runtime/src/model.cc (legacy strategy_search / optimize with
//    --budget, --alpha; Metropolis acceptance on simulated runtime)
//  * Unity: lib/compiler/src/unity_algorithm.cc:27-91 (intended body):
//    priority queue of GraphOptimizeState{pcg, mapping, runtime}; prune states
//    worse than best * alpha; expand every substitution at every match;
//    keep states with runtime <= threshold and #ops <= max_num_ops; `budget`
//    expansions; state identity = structural graph equality
//    (graph_optimize_state.cc:10-47).
#pragma once
#include <map>
#include <string>

#include "ff/computation_graph.h"
#include "ff/machine.h"
#include "ff/mapping.h"
#include "ff/parallelize.h"
#include "ff/pipeline.h"
#include "ff/simulator.h"
#include "ff/substitution.h"

namespace ff {

struct SearchConfig {
  int world = 1;
  int budget = 1000;            // MCMC proposals / Unity expansions
  double alpha = 1.05;          // Unity: prune states slower than best * alpha
  double threshold = 1e30;      // Unity: drop states slower than this (seconds)
  int max_num_ops = 1 << 20;    // Unity: drop graphs with more operator nodes
  double mcmc_beta = 200.0;     // Metropolis: accept worse with exp(-beta * rel_delta)
  double group_move_prob = 0.6; // propose the same config for every layer of the same signature
  uint64_t seed = 0x5eed;
  double time_limit = 60.0;     // seconds
  // Unity cost of every state: its DP machine mapping (shared subtree cache)
  // simulated, against whole-world placements (false: whole-world only, the
  // mapping DP runs once on the winner -- final_machine_mapping)
  bool use_machine_mapping = true;
  double mapping_alpha = 1.2;   // map states whose whole-world cost <= best so far * this
  int max_mapped_states = 64;   // at most this many mappings per search (-1: no cap); the
                                // first states popped are the cheapest, so the cap keeps the
                                // mapping on the search's front
  // graph_optimize: Unity best-first pops (-1: `budget`, the reference's
  // single --budget drives the whole search, unity_algorithm.cc:37-90) and
  // the share of time_limit MCMC may use before Unity starts
  int unity_budget = -1;
  double mcmc_time_share = 0.5;
  // graph_optimize: run the machine-mapping DP once on the final PCG and keep
  // its placements when the simulator prices them below the whole-world ones
  bool final_machine_mapping = true;
  // graph_optimize: pipeline-parallel candidates (ff/pipeline.h) priced at
  // `micro_batches` micro-batches per optimizer step against the searched
  // strategy run on the same micro-batches; with 1 micro-batch a pipeline
  // can only idle (all costs are then per batch, as without it)
  bool pipeline = true;
  int micro_batches = 1;
  // rule set added to the built-in parallelization rules (legacy TASO corpus
  // JSON or a substitution-set JSON, load_substitutions); "" = none
  std::string substitution_path;
  SearchSpaceOptions space;
  SimConfig sim;
};

struct SearchResult {
  std::string algorithm;
  ParallelComputationGraph pcg;
  StrategyConfig strategy;               // MCMC only
  std::map<int, Placement> views;        // PCG node -> devices (empty: whole world)
  double cost = 0;                       // simulated seconds / iteration
  double data_parallel_cost = 0;
  double unmapped_cost = -1;             // graph_optimize: cost before the final mapping (-1: not run)
  int iterations = 0;
  int evaluated = 0;
  int accepted = 0;
  double elapsed = 0;
  bool time_limited = false;             // ended on SearchConfig::time_limit, not the budget
  Json trace;                            // [[iteration, best cost], ...]
  int rules = 0;                         // Unity: rules tried (built-in + rule set)
  int rule_set_rules = 0;                // Unity: of which from the rule set
  std::vector<std::string> best_rules;   // Unity: rewrites from the initial PCG to the best one
  int64_t mapping_cache_entries = 0;     // Unity joint search: shared mapping-cache size / hits
  int64_t mapping_cache_hits = 0;
  int mapped_states = 0;                 // states priced with their own machine mapping
  int pipeline_stages = 0;               // > 0: the pipeline plan won (views = stage blocks)
  int micro_batches = 1;                 // costs are per micro-batch of a step of this many
  Json pipeline = Json::array();         // every pipeline candidate priced
  Json memory_plan;                      // liveness memory plan of the winner (max over devices)
  Json to_json(const ComputationGraph* cg = nullptr) const;
};

// The rule set behind SearchConfig::substitution_path (loaded once per path).
const std::vector<Substitution>& cached_substitutions(const std::string& path);

// Cost of a lowered strategy with the simulator (inf if invalid).
double evaluate_strategy(const ComputationGraph& cg, const StrategyConfig& s, const CostModel& cm,
                         const SimConfig& sim, int world, SimResult* out = nullptr);

SearchResult mcmc_search(const ComputationGraph& cg, const CostModel& cm, const SearchConfig& cfg,
                         const StrategyConfig* initial = nullptr);
SearchResult unity_search(const ParallelComputationGraph& initial, const CostModel& cm, const SearchConfig& cfg,
                          const std::vector<Substitution>& extra_rules = {});
// MCMC from data parallel, then Unity refinement of the best PCG; returns the
// best of {data parallel, MCMC, Unity} by simulated iteration time.
SearchResult graph_optimize(const ComputationGraph& cg, const CostModel& cm, const SearchConfig& cfg);

// JSON forms of the configs (keys as in SearchConfig / SimConfig; "sim" nests).
SimConfig sim_config_from_json(const Json& j);
SearchConfig search_config_from_json(const Json& j);

}  // namespace ff
