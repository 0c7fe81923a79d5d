// Machine mapping: place every operator of a PCG on a MachineView by dynamic
// programming over its series-parallel decomposition.
//
// Parity (reference lib/compiler/src/compiler/machine_mapping/):
//  * MachineMappingProblemTree: leaves are unmapped op cost-estimate keys
//    (op attrs + input / weight / output parallel shapes), series splits carry
//    the AbstractedTensorSetMovement of the tensors crossing them, keyed by
//    the tree paths of their producer / consumer leaves
//    (machine_mapping_problem_tree/get_machine_mapping_problem_tree.cc:12-51,
//    abstracted_tensor_set_movement/get_abstracted_tensor_set_movement_across_split.cc:15-61)
//  * get_optimal_machine_mapping (get_optimal_machine_mapping.cc:27-252):
//    series split = every assignment of allowed machine views to the
//    boundary layers on each side, each side solved under those constraints,
//    total = pre + concretized movement cost + post; parallel split = the
//    better of both children in series on the full resources and every
//    resource split with cost = max; leaf = minimum over the allowed views
//    (or the one view the constraints fix); memoized on {subtree, resources,
//    constraints} (machine_mapping_cache.cc)
//  * MachineMappingConstraints (machine_mapping_constraints.cc:13-112),
//    series_combine / parallel_combine / minimize_runtime
//    (machine_mapping_result.cc:10-136), resource splits
//    (get_machine_resource_splits.cc:7-29)
//
// The DP is generic over a cost estimator (CostEstimator interface,
// cost_estimator.h:13-41) so the reference's fake-cost-table cases run
// unchanged (tests/test_machine_mapping.py).  For a PCG the estimator is the
// MI355X CostModel: a leaf costs its forward + backward (+ weight-gradient
// sync) on the view's devices, a movement the region-intersection transfers
// between the producer's and consumer's device sets.  Resources carry an
// offset so the children of a resource split get disjoint absolute devices,
// and the chosen views become device lists (`Placement`) the executor runs:
// strided views included.
//
// One difference: a boundary layer that an enclosing split already fixed is
// enumerated with that view only (the reference's with_additional_constraints
// would throw on the other assignments).
#pragma once
#include <functional>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/machine.h"
#include "ff/simulator.h"
#include "ff/sp.h"

namespace ff {

// ---------------------------------------------------------------------------
// problem tree
struct UnmappedOpKey {
  OpAttrs op;
  std::vector<ParallelTensorShape> inputs, weights, outputs;
  int node = -1;    // PCG node the leaf stands for (-1: synthetic problem)
  std::string id;   // identity of a synthetic leaf (tests)
  // the op's task space: its first output's degrees [shard..., sum, copy]
  std::vector<int> task_space() const;
};

struct AbstractedSingleTensorMovement {
  ParallelTensorShape shape;
  std::set<BinaryTreePath> src;  // producer leaves, relative to the split's left child
  std::set<BinaryTreePath> dst;  // consumer leaves, relative to the split's right child
};

struct MMProblemTree {
  enum Kind { LEAF = 0, SERIES = 1, PARALLEL = 2 };
  struct Entry {
    Kind kind = LEAF;
    int left = -1, right = -1;
    UnmappedOpKey leaf;
    std::vector<AbstractedSingleTensorMovement> movement;  // SERIES only
  };
  std::vector<Entry> e;
  int root = -1;
  int add_leaf(UnmappedOpKey k);
  int add_series(std::vector<AbstractedSingleTensorMovement> m, int l, int r);
  int add_parallel(int l, int r);
  std::vector<BinaryTreePath> leaf_paths(int idx) const;
  int subtree_at(int idx, const BinaryTreePath& path) const;  // -1 if invalid
  // content signature of every subtree (index -> 128-bit hex string): equal
  // signatures = identical leaves (op attrs, input / weight / output parallel
  // shapes, synthetic ids), split kinds and movements
  std::vector<std::string> signatures() const;
};

// A sub-machine: nodes [node_offset, +num_nodes) x GPUs [gpu_offset, +gpus_per_node).
struct MachineResource {
  int node_offset = 0, num_nodes = 1;
  int gpu_offset = 0, gpus_per_node = 1;
  int num_devices() const { return num_nodes * gpus_per_node; }
  bool operator==(const MachineResource& o) const {
    return node_offset == o.node_offset && num_nodes == o.num_nodes && gpu_offset == o.gpu_offset &&
           gpus_per_node == o.gpus_per_node;
  }
  bool operator<(const MachineResource& o) const;
  std::string str() const;
};
// Power-of-two node splits and GPUs-per-node splits, both orders.
std::vector<std::pair<MachineResource, MachineResource>> get_machine_resource_splits(const MachineResource& r);
// Allowed views of a task space on a sub-machine, in absolute coordinates.
std::vector<MachineView> get_allowed_machine_views(const std::vector<int>& task_space, const MachineResource& r,
                                                   const MachineSpecification& spec);

using ObliviousMapping = std::map<BinaryTreePath, MachineView>;  // ParallelLayerGuidObliviousMachineMapping

struct MachineMappingConstraints {
  std::map<BinaryTreePath, std::optional<MachineView>> views;
  std::string key() const;
};
MachineMappingConstraints get_unconstrained_solution_for_layers(const std::vector<BinaryTreePath>& layers);
MachineMappingConstraints restrict_to_child(const MachineMappingConstraints& c, int child);  // 0 left, 1 right
// nullopt when an assignment contradicts a view the constraints already fix
std::optional<MachineMappingConstraints> with_additional_constraints(const MachineMappingConstraints& c,
                                                                    const ObliviousMapping& extra);

struct FeasibleMachineMapping {
  double runtime = 0;
  ObliviousMapping mapping;
};
using MMResult = std::optional<FeasibleMachineMapping>;
MMResult series_combine(double comm, const MMResult& pre, const MMResult& post, bool r_then_l = false);
MMResult parallel_combine(const MMResult& l, const MMResult& r);
MMResult minimize_runtime(const MMResult& a, const MMResult& b);

struct SingleTensorMovement {
  ParallelTensorShape shape;
  std::vector<MachineView> src, dst;
  std::vector<std::vector<int>> src_task_spaces, dst_task_spaces;  // of the producer / consumer leaves
};

class MMCostEstimator {
 public:
  virtual ~MMCostEstimator() = default;
  virtual double estimate_op(const UnmappedOpKey& k, const MachineView& v) const = 0;
  virtual double estimate_movement(const std::vector<SingleTensorMovement>& m) const = 0;
};

struct MMContext {
  const MMCostEstimator* cost = nullptr;
  std::function<std::vector<MachineView>(const UnmappedOpKey&, const MachineResource&)> allowed_views;
  size_t max_boundary_assignments = 4096;  // cap on one side's boundary view assignments
};

// Memo of solved subproblems.  Keys name a subtree by its CONTENT (a
// signature of its leaves' op attrs + parallel shapes, its splits and their
// movements: MMProblemTree::signatures), not by its index in one tree, so
// one cache can serve every PCG a search visits: a rewrite that changes a few
// operators leaves the other subtrees' entries valid (the reference's
// MachineMappingCache keyed by MachineMappingState, machine_mapping_cache.cc,
// shared across the states of unity_algorithm.cc:37-90).
struct MMCache {
  std::map<std::string, MMResult> results;
  size_t hits = 0, misses = 0;
};

MMResult get_optimal_machine_mapping(MMCache& cache, const MMContext& ctx, const MMProblemTree& tree, int idx,
                                     const MachineResource& resources, const MachineMappingConstraints& constraints);
// whole tree, unconstrained
MMResult get_optimal_machine_mapping(MMCache& cache, const MMContext& ctx, const MMProblemTree& tree,
                                     const MachineResource& resources);

// ---------------------------------------------------------------------------
// PCG adapter
struct PCGMappingProblem {
  MMProblemTree tree;
  std::map<BinaryTreePath, int> node_of_path;  // leaf path -> PCG node
};
PCGMappingProblem get_machine_mapping_problem_tree(const ParallelComputationGraph& pcg);

// Leaves: forward + backward (+ gradient sync) of the op on the view's
// devices; movements: region-intersection transfers (CostModel).
class PCGCostEstimator : public MMCostEstimator {
 public:
  PCGCostEstimator(const ParallelComputationGraph& pcg, const CostModel& cm, bool include_sync = true)
      : pcg_(pcg), cm_(cm), include_sync_(include_sync) {}
  double estimate_op(const UnmappedOpKey& k, const MachineView& v) const override;
  double estimate_movement(const std::vector<SingleTensorMovement>& m) const override;

 private:
  const ParallelComputationGraph& pcg_;
  const CostModel& cm_;
  bool include_sync_;
};

struct MachineMappingResult {
  double runtime = 0;                          // estimated seconds / iteration (no overlap)
  bool feasible = true;
  std::map<int, Placement> views;              // PCG node -> devices (task linear order)
  std::map<int, MachineView> machine_views;    // PCG node -> view (data-path nodes)
  size_t cache_entries = 0;
  Json to_json() const;
};

struct MachineMappingOptions {
  bool include_sync = true;
  // views the executor's canonical placement produces from a device block
  // (stride-1 intra-node views) only; false: every allowed (strided) view
  bool contiguous_only = false;
};

// `shared`: a cache reused across calls (a search's states); null = private
MachineMappingResult get_optimal_machine_mapping(const ParallelComputationGraph& pcg, const CostModel& cm, int world,
                                                 const MachineMappingOptions& opt = {}, MMCache* shared = nullptr);

}  // namespace ff
