// Machine mapping: place every operator of a PCG on a device block by
// dynamic programming over its series-parallel decomposition.
//
// Parity: compiler/machine_mapping/get_optimal_machine_mapping.cc:27-252
// (series: pre + comm + post; parallel: min(serial on the full machine,
// max over resource splits); leaf: min over allowed views; memoized on
// {subtree, resources}), machine_mapping_result.cc:10-136,
// get_machine_mapping_problem_tree.cc:12-51 (leaves carry the op attrs and
// parallel shapes), abstracted tensor-set movement across series splits.
//
// MI355X-first choices: candidate views are aligned device blocks (the
// executor's canonical layouts; xGMI is all-to-all inside a node so block
// position only matters for movement), leaves are costed with the analytic
// / profiled CostModel, and the series split prices the tensors crossing it
// with the concrete placements chosen on both sides (left and right are
// solved independently and the movement is added; the reference enumerates
// boundary-view constraints instead — with aligned blocks the unconstrained
// optimum of each side is a full-resource block in all but pathological
// cases, so the two agree and this is O(tree x blocks)).
#pragma once
#include <map>

#include "ff/computation_graph.h"
#include "ff/machine.h"
#include "ff/simulator.h"
#include "ff/sp.h"

namespace ff {

struct MachineMappingResult {
  double runtime = 0;                 // estimated seconds / iteration (no overlap)
  std::map<int, DeviceBlock> views;   // PCG node -> block
  bool feasible = true;
  Json to_json() const;
};

struct MachineMappingContext {
  const CostModel* cost = nullptr;
  bool allow_sub_blocks = true;  // leaves may use aligned sub-blocks of their resource
  bool include_sync = true;
};

class MachineMapper {
 public:
  MachineMapper(const ParallelComputationGraph& pcg, MachineMappingContext ctx);
  MachineMappingResult solve(const DeviceBlock& resources);
  const SPTree& tree() const { return tree_; }
  size_t cache_size() const { return cache_.size(); }

 private:
  MachineMappingResult solve_node(int idx, const DeviceBlock& res);
  MachineMappingResult leaf(int node, const DeviceBlock& res);
  double movement(const std::vector<int>& left_leaves, const std::vector<int>& right_leaves,
                  const MachineMappingResult& l, const MachineMappingResult& r);
  const ParallelComputationGraph& pcg_;
  MachineMappingContext ctx_;
  std::map<int, NodeRole> roles_;
  SPTree tree_;
  std::map<std::pair<int, DeviceBlock>, MachineMappingResult> cache_;
  std::map<int, std::vector<int>> leaves_of_;
};

// Convenience: optimal mapping of `pcg` on devices [0, world).
MachineMappingResult get_optimal_machine_mapping(const ParallelComputationGraph& pcg, const CostModel& cm,
                                                 int world);

}  // namespace ff
