#include "ff/simulator.h"

#include <algorithm>
#include <sstream>

namespace ff {

std::map<int, NodeRole> classify_nodes(const ParallelComputationGraph& pcg) {
  std::map<int, NodeRole> r;
  for (int id : pcg.g.topo_order()) {
    auto const& n = pcg.g.node(id);
    auto t = n.label.op.type;
    if (t == OpType::WEIGHT) r[id] = NodeRole::WEIGHT_PATH;
    else if (t == OpType::INPUT) r[id] = NodeRole::INPUT_PATH;
    else if (is_parallel_op(t)) {
      auto in = r.at(n.inputs.at(0).node);
      r[id] = (in == NodeRole::WEIGHT_PATH || in == NodeRole::INPUT_PATH) ? in : NodeRole::PARALLEL;
    } else {
      r[id] = NodeRole::COMPUTE;
    }
  }
  return r;
}

OpCost pcg_node_cost(const CostModel& cm, const ParallelComputationGraph& pcg, int node, int block_size) {
  auto const& n = pcg.g.node(node);
  auto t = n.label.op.type;
  if (t == OpType::INPUT || t == OpType::WEIGHT || t == OpType::NOOP) return OpCost{};
  std::vector<ParallelTensorShape> outs;
  for (auto const& o : n.outputs) outs.push_back(o.shape);
  if (is_parallel_op(t)) return cm.parallel_op_cost(n.label.op, pcg.shape(n.inputs.at(0)), outs.at(0), block_size);
  std::vector<ParallelTensorShape> ins, ws;
  for (auto const& v : pcg.layer_data_inputs(node)) ins.push_back(pcg.shape(v));
  for (auto const& v : pcg.layer_weights(node)) ws.push_back(pcg.shape(v));
  return cm.op_cost(n.label.op, ins, ws, outs, block_size);
}

DiGraph data_path_digraph(const ParallelComputationGraph& pcg) {
  auto roles = classify_nodes(pcg);
  DiGraph g;
  for (auto const& kv : roles)
    if (kv.second != NodeRole::WEIGHT_PATH) g.add_node(kv.first);
  for (int id : pcg.g.node_ids()) {
    if (roles.at(id) == NodeRole::WEIGHT_PATH) continue;
    for (auto const& v : pcg.g.node(id).inputs)
      if (roles.at(v.node) != NodeRole::WEIGHT_PATH) g.add_edge(v.node, id);
  }
  return g;
}

Json SimResult::to_json() const {
  Json j = Json::object();
  j["iteration_time"] = iteration_time;
  j["forward_time"] = forward_time;
  j["backward_end"] = backward_end;
  j["sync_time"] = sync_time;
  j["exposed_sync"] = exposed_sync;
  j["update_time"] = update_time;
  j["comm_time"] = comm_time;
  j["peak_memory"] = peak_memory;
  j["memory_penalty"] = memory_penalty;
  j["num_tasks"] = num_tasks;
  return j;
}

namespace {

struct Dep {
  int task;
  double xfer;
};

struct TaskRec {
  SimTask t;
  std::vector<Dep> deps;
  bool comm_lane = false;
};

}  // namespace

SimResult Simulator::simulate(const ParallelComputationGraph& pcg, const std::map<int, DeviceBlock>& views,
                              bool keep_tasks) const {
  const int world = std::max(1, cfg_.world);
  auto const& spec = cm_.spec();
  auto roles = classify_nodes(pcg);
  auto order = pcg.g.topo_order();
  auto block_of = [&](int n) {
    auto it = views.find(n);
    return it == views.end() ? DeviceBlock{0, world} : it->second;
  };
  std::map<int, std::vector<int>> consumers;
  for (int id : order)
    for (auto const& v : pcg.g.node(id).inputs) consumers[v.node].push_back(id);

  std::vector<TaskRec> tasks;
  std::map<int, int> fwd, bwd;
  std::map<int, OpCost> cost;
  SimResult res;
  bool any_sync = false;
  for (int id : order) {
    auto role = roles.at(id);
    if (role != NodeRole::COMPUTE && role != NodeRole::PARALLEL) continue;
    auto b = block_of(id);
    cost[id] = pcg_node_cost(cm_, pcg, id, b.size);
    if (cost[id].sync > 0) any_sync = true;
  }
  const double bwd_scale = (cfg_.overlap_grad_sync && any_sync) ? 1.0 + cfg_.comm_compute_slowdown : 1.0;
  // forward tasks (executor order = topological order)
  for (int id : order) {
    auto role = roles.at(id);
    if (role != NodeRole::COMPUTE && role != NodeRole::PARALLEL) continue;
    auto b = block_of(id);
    TaskRec r;
    r.t.type = role == NodeRole::PARALLEL ? SimTask::COMM : SimTask::FORWARD;
    r.t.node = id;
    r.t.name = pcg.g.node(id).label.name + ":fwd";
    r.t.dev_start = b.start;
    r.t.dev_size = b.size;
    r.t.run_time = cost[id].forward;
    if (role == NodeRole::PARALLEL) res.comm_time += cost[id].forward;
    for (auto const& v : pcg.g.node(id).inputs) {
      auto it = fwd.find(v.node);
      if (it == fwd.end()) continue;
      auto pb = block_of(v.node);
      double x = (pb == b) ? 0.0 : cm_.movement_cost(pcg.shape(v), pb, b);
      r.deps.push_back({it->second, x});
    }
    fwd[id] = static_cast<int>(tasks.size());
    tasks.push_back(std::move(r));
  }
  // backward tasks (reverse topological order), gradient buckets
  struct Bucket {
    double bytes = 0;
    int copy = 1;
    DeviceBlock block;
    int last_task = -1;
  };
  std::map<std::pair<DeviceBlock, int>, Bucket> buckets;
  std::map<DeviceBlock, double> params_per_block;  // local params (for the update)
  std::map<DeviceBlock, std::vector<int>> sync_tasks_of_block;
  std::vector<int> pending_sync;  // buckets flushed after backward when not overlapping
  auto emit_allreduce = [&](Bucket& bk, int after_task) {
    if (bk.bytes <= 0) return;
    TaskRec r;
    r.t.type = SimTask::ALLREDUCE;
    r.t.name = "allreduce";
    r.t.dev_start = bk.block.start;
    r.t.dev_size = bk.block.size;
    r.t.run_time = CollectiveCost::all_reduce(bk.bytes, bk.copy, spec);
    res.sync_time += r.t.run_time;
    r.comm_lane = true;
    r.deps.push_back({after_task, 0.0});
    sync_tasks_of_block[bk.block].push_back(static_cast<int>(tasks.size()));
    tasks.push_back(std::move(r));
    bk.bytes = 0;
  };
  int last_bwd = -1;
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    int id = *it;
    auto role = roles.at(id);
    if (role != NodeRole::COMPUTE && role != NodeRole::PARALLEL) continue;
    auto b = block_of(id);
    TaskRec r;
    r.t.type = role == NodeRole::PARALLEL ? SimTask::COMM : SimTask::BACKWARD;
    r.t.node = id;
    r.t.name = pcg.g.node(id).label.name + ":bwd";
    r.t.dev_start = b.start;
    r.t.dev_size = b.size;
    r.t.run_time = cost[id].backward * (role == NodeRole::COMPUTE ? bwd_scale : 1.0);
    if (role == NodeRole::PARALLEL) res.comm_time += cost[id].backward;
    r.deps.push_back({fwd.at(id), 0.0});
    for (int c : consumers[id]) {
      auto jt = bwd.find(c);
      if (jt == bwd.end()) continue;
      auto cb = block_of(c);
      double x = (cb == b) ? 0.0 : cm_.movement_cost(pcg.shape({id, 0}), cb, b);
      r.deps.push_back({jt->second, x});
    }
    int tid = static_cast<int>(tasks.size());
    bwd[id] = tid;
    tasks.push_back(std::move(r));
    last_bwd = tid;
    if (role != NodeRole::COMPUTE) continue;
    auto const& node = pcg.g.node(id);
    auto ws = pcg.layer_weights(id);
    for (size_t wi = 0; wi < ws.size(); ++wi) {
      auto const& ps = pcg.shape(ws[wi]);
      double elems = static_cast<double>(ps.piece_shape().num_elements());
      params_per_block[b] += elems;
      if (ps.discard_copy_degree <= 1) continue;
      bool gemm_w = wi == 0 && (node.label.op.type == OpType::LINEAR ||
                                node.label.op.type == OpType::MULTIHEAD_ATTENTION);
      double bytes = elems * ((cfg_.bf16_weight_grads && gemm_w) ? 2.0 : 4.0);
      auto key = std::make_pair(b, ps.discard_copy_degree);
      auto& bk = buckets[key];
      bk.copy = ps.discard_copy_degree;
      bk.block = b;
      bk.bytes += bytes;
      bk.last_task = tid;
      if (cfg_.overlap_grad_sync && bk.bytes >= cfg_.bucket_bytes) emit_allreduce(bk, tid);
    }
  }
  for (auto& kv : buckets) emit_allreduce(kv.second, last_bwd >= 0 ? last_bwd : kv.second.last_task);
  // optimizer update per device block, after its gradient sync
  if (cfg_.include_update) {
    for (auto const& kv : params_per_block) {
      TaskRec r;
      r.t.type = SimTask::UPDATE;
      r.t.name = "update";
      r.t.dev_start = kv.first.start;
      r.t.dev_size = kv.first.size;
      r.t.run_time = kv.second * cfg_.update_bytes_per_param / spec.hbm_bandwidth + 2 * spec.kernel_launch_overhead;
      res.update_time = std::max(res.update_time, r.t.run_time);
      if (last_bwd >= 0) r.deps.push_back({last_bwd, 0.0});
      for (int s : sync_tasks_of_block[kv.first]) r.deps.push_back({s, 0.0});
      tasks.push_back(std::move(r));
    }
  }
  // list scheduling in creation order (= each rank's issue order)
  std::vector<double> comp_free(world + 64, 0.0), comm_free(world + 64, 0.0);
  double end = 0, fwd_end = 0, bwd_end = 0;
  for (auto& r : tasks) {
    double ready = 0;
    for (auto const& d : r.deps) ready = std::max(ready, tasks[d.task].t.end_time + d.xfer);
    auto& lane = r.comm_lane ? comm_free : comp_free;
    double start = ready;
    int lo = std::max(0, r.t.dev_start), hi = std::min(static_cast<int>(lane.size()), r.t.dev_start + r.t.dev_size);
    for (int d = lo; d < hi; ++d) start = std::max(start, lane[d]);
    r.t.ready_time = ready;
    r.t.start_time = start;
    r.t.end_time = start + r.t.run_time;
    for (int d = lo; d < hi; ++d) lane[d] = r.t.end_time;
    end = std::max(end, r.t.end_time);
    if (r.t.type == SimTask::FORWARD || (r.t.type == SimTask::COMM && r.t.name.size() > 4 &&
                                         r.t.name.compare(r.t.name.size() - 4, 4, ":fwd") == 0))
      fwd_end = std::max(fwd_end, r.t.end_time);
    if (r.t.type == SimTask::BACKWARD || (r.t.type == SimTask::COMM && r.t.name.size() > 4 &&
                                          r.t.name.compare(r.t.name.size() - 4, 4, ":bwd") == 0))
      bwd_end = std::max(bwd_end, r.t.end_time);
  }
  // memory per device
  std::vector<double> mem(world, 0.0);
  for (auto const& kv : cost) {
    auto b = block_of(kv.first);
    for (int d = std::max(0, b.start); d < std::min(world, b.start + b.size); ++d) mem[d] += kv.second.memory;
  }
  res.peak_memory = mem.empty() ? 0.0 : *std::max_element(mem.begin(), mem.end());
  if (res.peak_memory > spec.hbm_capacity)
    res.memory_penalty = (res.peak_memory - spec.hbm_capacity) / 1e6 * cfg_.memory_penalty_per_mb;
  res.forward_time = fwd_end;
  res.backward_end = bwd_end;
  res.iteration_time = end + res.memory_penalty;
  res.exposed_sync = std::max(0.0, end - bwd_end - res.update_time);
  res.num_tasks = static_cast<int>(tasks.size());
  if (keep_tasks)
    for (auto& r : tasks) {
      for (auto const& d : r.deps) r.t.deps.push_back(d.task);
      res.tasks.push_back(r.t);
    }
  return res;
}

std::string Simulator::task_graph_dot(const SimResult& r) const {
  static const char* kind[] = {"FWD", "BWD", "COMM", "UPDATE", "ALLREDUCE"};
  static const char* color[] = {"lightblue", "lightsalmon", "khaki", "palegreen", "plum"};
  std::ostringstream os;
  os << "digraph taskgraph {\n  node [shape=box, style=filled];\n";
  for (size_t i = 0; i < r.tasks.size(); ++i) {
    auto const& t = r.tasks[i];
    os << "  t" << i << " [label=\"" << t.name << "\\n" << kind[t.type] << " dev[" << t.dev_start << ","
       << t.dev_start + t.dev_size << ")\\n" << t.run_time * 1e3 << " ms @ " << t.start_time * 1e3
       << "\", fillcolor=" << color[t.type] << "];\n";
  }
  for (size_t i = 0; i < r.tasks.size(); ++i)
    for (int d : r.tasks[i].deps) os << "  t" << d << " -> t" << i << ";\n";
  os << "}\n";
  return os.str();
}

}  // namespace ff
