// Event-driven simulator of one training iteration of a PCG on a machine.
//
// Parity: lib/runtime/src/simulator.cc Simulator::simulate_runtime (:816-1243)
// and LogicalTaskgraphBasedSimulator (:1245-1870):
//  * per-operator forward / backward tasks on the devices of the operator's
//    placement (each device's compute lane runs its partition; :823-841);
//  * data dependencies between operators on different device sets become
//    transfer tasks sized by the intersection of the producer's and the
//    consumer's pieces (region intersection, :843-899), from a holder of the
//    piece to every consumer device that lacks it; with a NetworkModel the
//    transfer is routed and occupies every link of its route
//    (route_transfer, :1482-1683), else its device pair's xGMI link;
//  * weight-gradient synchronization: NCCL mode = bucketed all-reduces on
//    each device's communication lane, serialized per device and overlapped
//    with the rest of the backward pass (the NCCL pass, :1087-1215; with a
//    NetworkModel the all-reduce is priced by its ring expansion over the
//    routed links, expand_allreduce :1684-1795); parameter-server mode =
//    gradients reduced into the group leader, the update on the leader, the
//    weights broadcast back (barrier / update / final tasks, :957-1019);
//  * list scheduling in each rank's issue order with per-device (and
//    per-link) serialization (:1020-1085);
//  * framebuffer memory penalty (:1216-1242); dot export (--taskgraph).
//
// MI355X model: each device has a compute lane (one HIP stream: kernels and
// the inline RCCL collectives of parallel ops) and a communication lane (the
// bucketed gradient all-reduce stream the executor overlaps with backward).
// Gradient buckets mirror Executor's (grad dtype bf16 for GEMM weights), and
// the fused Adam/SGD update runs after each device's last bucket.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/machine.h"

namespace ff {

class NetworkModel;

struct SimConfig {
  int world = 1;                      // devices used by the executor
  bool overlap_grad_sync = true;
  double bucket_bytes = 64.0 * (1 << 20);
  bool include_update = true;
  double update_bytes_per_param = 30.0;  // fused Adam: w,m,v r/w + grad + bf16 copy
  double memory_penalty_per_mb = 1e-3;   // seconds per MB over capacity (reference: 1 ms / MB)
  double comm_compute_slowdown = 0.05;   // compute slowdown while a collective overlaps
  bool bf16_weight_grads = true;
  bool parameter_server = false;         // ParamSync::PS instead of all-reduce
  // row-sparse embedding update (the executor's sparse SGD): an EMBEDDING
  // table's update touches only the rows its indices name, not the table
  bool sparse_embedding_update = false;
  // the executor's kernel fusions (runtime/executor.py): an EW_ADD whose sum
  // feeds a LAYERNORM on the same devices runs inside the norm
  // (FUSED_ADD_LAYERNORM), and the graph's final SOFTMAX runs inside the
  // softmax + cross-entropy loss kernel (one read of the logits, one write of
  // their gradient, no separate backward)
  bool executor_fusions = true;
  const NetworkModel* network = nullptr; // routed transfers / collectives (LogicalTaskgraph mode)
};

struct SimTask {
  enum Type { FORWARD = 0, BACKWARD = 1, COMM = 2, UPDATE = 3, ALLREDUCE = 4, XFER = 5, REDUCE = 6, BCAST = 7,
              BARRIER = 8 };
  Type type = FORWARD;
  int node = -1;
  std::string name;
  int dev_start = 0, dev_size = 1;  // range covering `devices` (reports)
  std::vector<int> devices;         // lanes the task occupies
  std::vector<int> links;           // routed transfers: network link ids
  int src = -1, dst = -1;           // XFER endpoints
  double bytes = 0;
  double run_time = 0, ready_time = 0, start_time = 0, end_time = 0;
  std::vector<int> deps;
  double xfer = 0;
};

struct SimResult {
  double iteration_time = 0;   // seconds
  double forward_time = 0;     // critical-path forward end
  double backward_end = 0;
  double sync_time = 0;        // summed all-reduce / PS time
  double exposed_sync = 0;     // iteration_time - backward_end - update
  double update_time = 0;
  double comm_time = 0;        // summed parallel-op communication
  double xfer_time = 0;        // summed region-intersection transfer time
  double xfer_bytes = 0;
  double peak_memory = 0;      // max bytes on one device
  double memory_penalty = 0;
  int num_tasks = 0;
  int num_xfers = 0;
  std::vector<SimTask> tasks;  // only filled when keep_tasks
  Json to_json() const;
};

class Simulator {
 public:
  Simulator(const CostModel& cm, SimConfig cfg) : cm_(cm), cfg_(std::move(cfg)) {}
  const SimConfig& config() const { return cfg_; }
  // views: PCG node -> placement (device list in task order; default: the
  // whole world, devices 0..world-1)
  SimResult simulate(const ParallelComputationGraph& pcg, const std::map<int, Placement>& views = {},
                     bool keep_tasks = false) const;
  std::string task_graph_dot(const SimResult& r) const;

 private:
  const CostModel& cm_;
  SimConfig cfg_;
};

// Node classification shared by the simulator, the machine-mapping problem
// and the executor's folding rules.
enum class NodeRole { COMPUTE = 0, PARALLEL = 1, INPUT_PATH = 2, WEIGHT_PATH = 3 };
std::map<int, NodeRole> classify_nodes(const ParallelComputationGraph& pcg);
// Compute cost of a PCG node (op cost + its weights' gradient sync), per device.
OpCost pcg_node_cost(const CostModel& cm, const ParallelComputationGraph& pcg, int node, int block_size);
// The PCG data-flow DAG restricted to COMPUTE/PARALLEL/INPUT nodes.
DiGraph data_path_digraph(const ParallelComputationGraph& pcg);
// Region intersection of one tensor between two placements: (src device,
// dst device, bytes) for every consumer device that lacks its piece.
std::vector<std::tuple<int, int, double>> region_transfers(const ParallelTensorShape& t, const Placement& src,
                                                           const Placement& dst);

}  // namespace ff
