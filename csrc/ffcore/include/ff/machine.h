// Machine model: specification, machine views, resource splits, and the
// MI355X cost model (MFMA roofline + HBM3E + xGMI collectives).
//
// Parity:
//  * MachineSpecification{num_nodes, num_cpus_per_node, num_gpus_per_node,
//    inter/intra_node_bandwidth}: lib/pcg/include/pcg/machine_specification.struct.toml
//  * MachineView{start, dims[{stride, projection}]} + get_machine_space_coordinate:
//    lib/pcg/src/pcg/machine_view.cc:45-113
//  * allowed machine views: lib/compiler/src/compiler/allowed_machine_views.cc:24-120
//  * resource splits (power-of-two): get_machine_resource_splits.cc:7-29
//  * machine models (Simple/Enhanced/Networked): lib/runtime/src/machine_model.cc
//
// MI355X-first: 8 GPUs per node fully connected by xGMI (7 links each), so
// placement is topology-symmetric inside a node; candidate views are aligned
// power-of-two device blocks (start, size), which is what the executor's
// canonical layouts use.  Collectives are priced with a ring / direct model
// over the per-GPU xGMI bandwidth, calibratable from measured RCCL numbers.
#pragma once
#include <mutex>
#include <unordered_map>
#include <map>
#include <optional>
#include <string>
#include <vector>

#include "ff/json.h"
#include "ff/op_attrs.h"
#include "ff/types.h"

namespace ff {

struct MachineSpecification {
  int num_nodes = 1;
  int num_cpus_per_node = 1;
  int num_gpus_per_node = 8;
  double inter_node_bandwidth = 50e9;   // bytes/s per GPU (NIC)
  double intra_node_bandwidth = 300e9;  // bytes/s per GPU achievable RCCL bus bandwidth over xGMI
  // ---- MI355X device model
  double peak_bf16_flops = 2.5e15;      // dense MFMA
  double peak_fp32_flops = 157e12;
  double mfma_efficiency = 0.45;        // achieved fraction on large GEMMs (measured ~1.1 PF hipBLASLt)
  double hbm_bandwidth = 6.0e12;        // achievable (6.3 TB/s float4 copy)
  double hbm_capacity = 288e9;
  double kernel_launch_overhead = 4e-6; // s per kernel (graph-replayed ~1.5 us)
  double collective_latency = 8e-6;     // alpha per collective step
  // the executor computes in bf16 whatever dtype a tensor is declared with
  // (fp32 masters aside): analytic memory traffic counts 2 bytes per fp32
  // element (measured profile entries are used as they are)
  bool bf16_compute = true;
  int xgmi_links = 7;
  double xgmi_link_bandwidth = 64e9;    // per direction per link
  // Optional effective bus bandwidths (bytes/s) per group size p, from the
  // topology model (network.h NetworkModel::calibrate) or RCCL measurements;
  // override the analytic link model when present.
  std::map<int, double> collective_bw;
  std::map<int, double> all_to_all_bw;

  int num_devices() const { return num_nodes * num_gpus_per_node; }
  Json to_json() const;
  static MachineSpecification from_json(const Json& j);
  static MachineSpecification mi355x(int num_nodes = 1, int gpus_per_node = 8);
};

enum class ProjectionType { INTRA_NODE = 0, INTER_NODE = 1 };

struct MachineViewDimension {
  int stride = 1;
  ProjectionType projection = ProjectionType::INTRA_NODE;
  bool operator==(const MachineViewDimension& o) const { return stride == o.stride && projection == o.projection; }
};

struct MachineSpaceCoordinate {
  int node_idx = 0;
  int device_idx = 0;
  bool operator==(const MachineSpaceCoordinate& o) const {
    return node_idx == o.node_idx && device_idx == o.device_idx;
  }
};

struct MachineView {
  MachineSpaceCoordinate start;
  std::vector<MachineViewDimension> dims;
  bool operator==(const MachineView& o) const { return start == o.start && dims == o.dims; }
  bool operator!=(const MachineView& o) const { return !(*this == o); }
  bool operator<(const MachineView& o) const;
  std::string str() const;
  Json to_json() const;
  static MachineView from_json(const Json& j);
};

// The devices an operator (or a tensor) occupies, in task linear order:
// entry lin * reps + r holds task coordinate unravel(lin) (row-major over
// [shard degrees..., sum, copy]), redundant replica r.  A contiguous device
// block [start, start + size) is the placement {start, ..., start + size - 1}.
using Placement = std::vector<int>;

extern const double kMovementInfeasible;

// Task space of an operator = the degrees of its output [shard..., sum, copy].
std::vector<int> operator_task_space(const ParallelTensorShape& out);

// Maps a task coordinate to a machine coordinate (mixed radix per projection,
// first task dimension fastest); nullopt when the coordinate is outside the
// task space or lands outside the machine.
std::optional<MachineSpaceCoordinate> get_machine_space_coordinate(const std::vector<int>& task_space, const MachineView& view,
                                                    const std::vector<int>& coord,
                                                    const MachineSpecification& spec);
std::vector<int> get_device_ids(const std::vector<int>& task_space, const MachineView& view,
                                const MachineSpecification& spec);

// A view's dimensions without its start (start_invariant_machine_view.h).
struct StartInvariantMachineView {
  std::vector<MachineViewDimension> dims;
  bool operator==(const StartInvariantMachineView& o) const { return dims == o.dims; }
};
StartInvariantMachineView start_invariant_from_machine_view(const MachineView& v);
MachineView machine_view_from_start_invariant(const StartInvariantMachineView& s, const MachineSpaceCoordinate& start);
// offset of a task from the view's start (the coordinate of the view placed
// at (0, 0)); nullopt outside the task space or the machine
std::optional<MachineSpaceCoordinate> get_machine_space_offset(const std::vector<int>& task_space,
                                                               const StartInvariantMachineView& s,
                                                               const std::vector<int>& coord,
                                                               const MachineSpecification& spec);
// Every strided view (strides up to the machine size, every start, every
// projection) whose devices fit the machine (allowed_machine_views.cc).
std::vector<MachineView> get_allowed_machine_views(const std::vector<int>& task_space,
                                                   const MachineSpecification& spec);

// Aligned device block used by the executor: devices [start, start + size).
struct DeviceBlock {
  int start = 0;
  int size = 1;
  bool operator==(const DeviceBlock& o) const { return start == o.start && size == o.size; }
  bool operator<(const DeviceBlock& o) const { return start != o.start ? start < o.start : size < o.size; }
};
// Canonical MachineView of an operator with task space `ts` on block `b`
// (first task dimension strided by the implicit replica count).
MachineView block_machine_view(const std::vector<int>& ts, const DeviceBlock& b, const MachineSpecification& spec);
// Power-of-two splits of a block into two disjoint halves-or-quarters.
std::vector<std::pair<DeviceBlock, DeviceBlock>> get_resource_splits(const DeviceBlock& b);
Placement block_placement(const DeviceBlock& b);
Placement block_placement(int start, int size);
// the devices of a view, in task linear order (= get_device_ids)
Placement view_placement(const std::vector<int>& task_space, const MachineView& v, const MachineSpecification& spec);

// ---------------------------------------------------------------------------
// Cost model
struct CollectiveCost {
  static double all_reduce(double bytes, int p, const MachineSpecification& s);
  static double all_gather(double bytes_out, int p, const MachineSpecification& s);     // bytes of the gathered result
  static double reduce_scatter(double bytes_in, int p, const MachineSpecification& s);  // bytes of the full input
  static double all_to_all(double bytes, int p, const MachineSpecification& s);          // bytes per rank
  static double p2p(double bytes, const MachineSpecification& s);
};

struct OpCost {
  double forward = 0;   // seconds
  double backward = 0;
  double memory = 0;    // bytes resident per device (weights + grads + optimizer + activations)
  double workspace = 0; // transient bytes beyond `memory` while the op runs (measured peak)
  double sync = 0;      // weight-gradient all-reduce time
  bool measured = false; // forward / backward from a measured profile entry
};

// Optional measured-profile table: op signature -> {fwd_ms, bwd_ms} and, when
// the profiler tracked the allocator (the reference's TrackedAllocator in
// local_cost_estimator.cc:29-90), resident_mb (activations alive after the
// forward: outputs + saved tensors) and peak_mb (allocator peak over forward
// + backward), both above the op's inputs and weights
struct ProfileEntry {
  double fwd_ms = 0, bwd_ms = 0;
  double resident_mb = -1, peak_mb = -1;  // -1: not measured
};
class ProfileTable {
 public:
  void load_json(const Json& j);
  bool lookup(const std::string& key, double& fwd, double& bwd) const;
  const ProfileEntry* find(const std::string& key) const;
  void put(const std::string& key, double fwd, double bwd);
  void put(const std::string& key, const ProfileEntry& e) { table_[key] = e; }
  Json to_json() const;
  size_t size() const { return table_.size(); }

 private:
  std::map<std::string, ProfileEntry> table_;
};

class CostModel {
 public:
  explicit CostModel(MachineSpecification spec) : spec_(std::move(spec)) {}
  CostModel(const CostModel& o) : spec_(o.spec_), profiles_(o.profiles_) {}
  CostModel& operator=(const CostModel& o) {
    spec_ = o.spec_;
    profiles_ = o.profiles_;
    clear_memo();
    return *this;
  }
  const MachineSpecification& spec() const { return spec_; }
  // mutable access to the measured table invalidates the memoised costs
  ProfileTable& profiles() {
    clear_memo();
    return profiles_;
  }

  // Compute cost of one piece (per-device) of an operator.
  OpCost op_cost(const OpAttrs& op, const std::vector<ParallelTensorShape>& inputs,
                 const std::vector<ParallelTensorShape>& weights, const std::vector<ParallelTensorShape>& outputs,
                 int block_size) const;
  // Cost of a parallel operator (forward / backward communication).
  OpCost parallel_op_cost(const OpAttrs& op, const ParallelTensorShape& in, const ParallelTensorShape& out,
                          int block_size) const;
  // Moving a tensor between two device blocks of the same layout.
  double movement_cost(const ParallelTensorShape& t, const DeviceBlock& src, const DeviceBlock& dst) const;
  // Moving a tensor between two placements (region intersection: piece i is
  // held by every device of entries [i*reps, (i+1)*reps) on each side; a
  // consumer device that does not hold its piece receives it from a holder;
  // transfers between distinct device pairs run concurrently over their
  // own xGMI links, inter-node pairs over the NIC).
  double movement_cost(const ParallelTensorShape& t, const Placement& src, const Placement& dst) const;
  static std::string signature(const OpAttrs& op, const std::vector<TensorShape>& pieces);

 private:
  OpCost op_cost_uncached(const OpAttrs& op, const std::vector<ParallelTensorShape>& inputs,
                          const std::vector<ParallelTensorShape>& weights,
                          const std::vector<ParallelTensorShape>& outputs, int block_size) const;
  OpCost parallel_op_cost_uncached(const OpAttrs& op, const ParallelTensorShape& in, const ParallelTensorShape& out,
                                   int block_size) const;
  void clear_memo() const {
    std::lock_guard<std::mutex> lk(memo_mu_);
    memo_.clear();
  }
  double gemm_time(double flops, double bytes, double eff_hint) const;
  MachineSpecification spec_;
  ProfileTable profiles_;
  // (op, parallel shapes, block) -> cost: a search re-costs the same
  // operators in thousands of candidate graphs that differ in a few nodes
  mutable std::unordered_map<size_t, OpCost> memo_;
  mutable std::mutex memo_mu_;
};

}  // namespace ff
