#include "ff/simulator.h"

#include <algorithm>
#include <set>
#include <sstream>
#include <tuple>

#include "ff/network.h"

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

std::vector<std::tuple<int, int, double>> region_transfers(const ParallelTensorShape& t, const Placement& src,
                                                           const Placement& dst) {
  std::vector<std::tuple<int, int, double>> out;
  if (src == dst || src.empty() || dst.empty()) return out;
  const int T = std::max(1, t.total_parallel_degree());
  if (static_cast<int>(src.size()) % T || static_cast<int>(dst.size()) % T) return out;
  const int rs = static_cast<int>(src.size()) / T, rd = static_cast<int>(dst.size()) / T;
  const double piece = static_cast<double>(t.piece_shape().size_bytes());
  std::map<std::pair<int, int>, double> bytes;
  for (int i = 0; i < T; ++i)
    for (int r = 0; r < rd; ++r) {
      const int d = dst[i * rd + r];
      bool held = false;
      for (int q = 0; q < rs && !held; ++q) held = src[i * rs + q] == d;
      if (!held) bytes[{src[i * rs + (r % rs)], d}] += piece;
    }
  for (auto const& kv : bytes) out.emplace_back(kv.first.first, kv.first.second, kv.second);
  return out;
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
  j["xfer_time"] = xfer_time;
  j["xfer_bytes"] = xfer_bytes;
  j["peak_memory"] = peak_memory;
  j["memory_penalty"] = memory_penalty;
  j["num_tasks"] = num_tasks;
  j["num_xfers"] = num_xfers;
  return j;
}

namespace {

std::vector<int> devset(const Placement& p) {
  std::vector<int> d = p;
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  return d;
}

enum Lane { COMPUTE_LANE = 0, COMM_LANE = 1 };

struct Rec {
  SimTask t;
  Lane lane = COMPUTE_LANE;
  std::vector<std::pair<int, double>> deps;  // (task, extra latency)
};

}  // namespace

SimResult Simulator::simulate(const ParallelComputationGraph& pcg, const std::map<int, Placement>& views,
                              bool keep_tasks) const {
  const int world = std::max(1, cfg_.world);
  auto const& spec = cm_.spec();
  const int gpn = std::max(1, spec.num_gpus_per_node);
  auto roles = classify_nodes(pcg);
  auto order = pcg.g.topo_order();
  const int n_ids = pcg.g.next_id();
  const Placement all = block_placement(0, world);
  auto place = [&](int n) -> const Placement& {
    auto it = views.find(n);
    return it == views.end() ? all : it->second;
  };
  auto active = [&](int id) {
    auto r = roles.at(id);
    return r == NodeRole::COMPUTE || r == NodeRole::PARALLEL;
  };
  std::vector<std::vector<int>> consumers(n_ids);
  for (int id : order)
    for (auto const& v : pcg.g.node(id).inputs) consumers[v.node].push_back(id);

  SimResult res;
  std::vector<OpCost> cost(n_ids);
  bool any_sync = false;
  for (int id : order) {
    if (!active(id)) continue;
    cost[id] = pcg_node_cost(cm_, pcg, id, static_cast<int>(place(id).size()));
    if (cost[id].sync > 0) any_sync = true;
  }
  if (cfg_.executor_fusions) {
    const double bw = spec.hbm_bandwidth;
    for (int id : order) {
      if (!active(id) || roles.at(id) != NodeRole::COMPUTE) continue;
      auto const& nd = pcg.g.node(id);
      const OpType t = nd.label.op.type;
      if (t == OpType::LAYERNORM) {
        auto ins = pcg.layer_data_inputs(id);
        if (ins.size() != 1) continue;
        const int p = ins[0].node;
        if (roles.at(p) != NodeRole::COMPUTE || pcg.g.node(p).label.op.type != OpType::EW_ADD) continue;
        if (place(p) != place(id)) continue;
        auto const& pin = pcg.layer_data_inputs(p);
        if (pin.size() != 2 || !(pcg.shape(pin[0]) == pcg.shape(ins[0])) || !(pcg.shape(pin[1]) == pcg.shape(ins[0])))
          continue;
        // the add runs inside the norm: one more input read, plus the sum
        // written out when something else also reads it (pre-LN residual)
        if (!cost[id].measured) {
          const double piece = static_cast<double>(pcg.shape(ins[0]).piece_shape().size_bytes());
          cost[id].forward += piece / bw * (consumers[p].size() > 1 ? 2.0 : 1.0);
        }
        const double sync = cost[p].sync;
        cost[p] = OpCost{};
        cost[p].sync = sync;
      } else if (t == OpType::SOFTMAX && consumers[id].empty() && !cost[id].measured) {
        const double piece = static_cast<double>(nd.outputs.at(0).shape.piece_shape().size_bytes());
        cost[id].forward = 2.0 * piece / bw + spec.kernel_launch_overhead;
        cost[id].backward = 0.0;
      }
    }
  }
  const double bwd_scale = (cfg_.overlap_grad_sync && any_sync) ? 1.0 + cfg_.comm_compute_slowdown : 1.0;

  std::vector<Rec> tasks;
  auto push = [&](SimTask::Type type, int node, std::string name, std::vector<int> devs, double run,
                  Lane lane) -> int {
    Rec r;
    r.t.type = type;
    r.t.node = node;
    r.t.name = std::move(name);
    r.t.devices = std::move(devs);
    if (!r.t.devices.empty()) {
      r.t.dev_start = r.t.devices.front();
      r.t.dev_size = r.t.devices.back() - r.t.devices.front() + 1;
    }
    r.t.run_time = run;
    r.lane = lane;
    tasks.push_back(std::move(r));
    return static_cast<int>(tasks.size()) - 1;
  };
  // region-intersection transfers of one tensor (forward activation or
  // backward gradient), after task `after`
  auto transfers = [&](const ParallelTensorShape& shp, const Placement& src, const Placement& dst, int after,
                       const std::string& name) {
    std::vector<int> ids;
    for (auto const& x : region_transfers(shp, src, dst)) {
      const int s = std::get<0>(x), d = std::get<1>(x);
      const double bytes = std::get<2>(x);
      double run;
      std::vector<int> links;
      if (cfg_.network && s < cfg_.network->topology().num_devices && d < cfg_.network->topology().num_devices) {
        auto const& rts = cfg_.network->routes(s, d);
        if (!rts.empty()) links = rts.front();
        run = cfg_.network->p2p_time(s, d, bytes);
      } else {
        const bool inter = s / gpn != d / gpn;
        run = bytes / (inter ? spec.inter_node_bandwidth : spec.xgmi_link_bandwidth) + spec.collective_latency;
      }
      int k = push(SimTask::XFER, -1, name, {s, d}, run, COMPUTE_LANE);
      tasks[k].t.src = s;
      tasks[k].t.dst = d;
      tasks[k].t.bytes = bytes;
      tasks[k].t.links = std::move(links);
      if (after >= 0) tasks[k].deps.push_back({after, 0.0});
      res.xfer_time += run;
      res.xfer_bytes += bytes;
      ++res.num_xfers;
      ids.push_back(k);
    }
    return ids;
  };

  // ---- forward (executor order = topological order)
  std::vector<int> fwd(n_ids, -1), bwd(n_ids, -1);
  for (int id : order) {
    if (!active(id)) continue;
    const bool par = roles.at(id) == NodeRole::PARALLEL;
    const Placement& P = place(id);
    std::vector<int> devs = P;
    std::vector<std::pair<int, double>> deps;
    for (auto const& v : pcg.g.node(id).inputs) {
      const int p = v.node;
      if (fwd[p] < 0) continue;
      const Placement& Pp = place(p);
      if (par) {
        // the redistribution collective runs over both placements
        devs.insert(devs.end(), Pp.begin(), Pp.end());
        deps.push_back({fwd[p], 0.0});
      } else if (Pp == P) {
        deps.push_back({fwd[p], 0.0});
      } else {
        auto xs = transfers(pcg.shape(v), Pp, P, fwd[p], pcg.g.node(id).label.name + ":in");
        if (xs.empty()) deps.push_back({fwd[p], 0.0});
        for (int x : xs) deps.push_back({x, 0.0});
      }
    }
    int k = push(par ? SimTask::COMM : SimTask::FORWARD, id, pcg.g.node(id).label.name + ":fwd", devset(devs),
                 cost[id].forward, COMPUTE_LANE);
    tasks[k].deps = std::move(deps);
    if (par) res.comm_time += cost[id].forward;
    fwd[id] = k;
  }

  // ---- backward (reverse topological order) + gradient synchronization
  struct Bucket {
    double bytes = 0;
    int copy = 1;
    std::vector<int> devs;
    int last_task = -1;
  };
  std::map<std::pair<std::vector<int>, int>, Bucket> buckets;
  std::vector<double> params_on(world + 64, 0.0);
  std::vector<int> last_bwd_on(world + 64, -1);
  std::map<int, std::vector<int>> sync_on;  // device -> sync tasks touching it
  std::vector<int> ps_final;                // PS broadcast tasks
  auto emit_allreduce = [&](Bucket& bk, int after) {
    if (bk.bytes <= 0) return;
    double run = CollectiveCost::all_reduce(bk.bytes, bk.copy, spec);
    if (cfg_.network && bk.copy > 1 && static_cast<int>(bk.devs.size()) >= bk.copy) {
      std::vector<int> g(bk.devs.begin(), bk.devs.begin() + bk.copy);
      bool ok = true;
      for (int d : g) ok = ok && d < cfg_.network->topology().num_devices;
      if (ok) run = cfg_.network->all_reduce_time(g, bk.bytes);
    }
    int k = push(SimTask::ALLREDUCE, -1, "allreduce", bk.devs, run, COMM_LANE);
    tasks[k].t.bytes = bk.bytes;
    tasks[k].deps.push_back({after, 0.0});
    res.sync_time += run;
    for (int d : bk.devs) sync_on[d].push_back(k);
    bk.bytes = 0;
  };
  int last_bwd = -1;
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    const int id = *it;
    if (!active(id)) continue;
    const bool par = roles.at(id) == NodeRole::PARALLEL;
    const Placement& P = place(id);
    std::vector<std::pair<int, double>> deps{{fwd[id], 0.0}};
    for (int c : consumers[id]) {
      if (bwd[c] < 0) continue;
      const Placement& Pc = place(c);
      if (par || roles.at(c) == NodeRole::PARALLEL || Pc == P) {
        deps.push_back({bwd[c], 0.0});
        continue;
      }
      bool any = false;
      for (auto const& v : pcg.g.node(c).inputs) {
        if (v.node != id) continue;
        for (int x : transfers(pcg.shape(v), Pc, P, bwd[c], pcg.g.node(id).label.name + ":grad")) {
          deps.push_back({x, 0.0});
          any = true;
        }
      }
      if (!any) deps.push_back({bwd[c], 0.0});
    }
    int k = push(par ? SimTask::COMM : SimTask::BACKWARD, id, pcg.g.node(id).label.name + ":bwd", tasks[fwd[id]].t.devices,
                 cost[id].backward * (par ? 1.0 : bwd_scale), COMPUTE_LANE);
    tasks[k].deps = std::move(deps);
    if (par) res.comm_time += cost[id].backward;
    bwd[id] = k;
    last_bwd = k;
    const auto ds = devset(P);
    for (int d : ds)
      if (d < static_cast<int>(last_bwd_on.size())) last_bwd_on[d] = k;
    if (par) continue;
    auto const& node = pcg.g.node(id);
    auto ws = pcg.layer_weights(id);
    for (size_t wi = 0; wi < ws.size(); ++wi) {
      auto const& ps = pcg.shape(ws[wi]);
      const double elems = static_cast<double>(ps.piece_shape().num_elements());
      double upd = elems;
      if (cfg_.sparse_embedding_update && node.label.op.type == OpType::EMBEDDING && wi == 0) {
        // rows named by this piece's indices x row width
        auto const& ip = pcg.shape(pcg.layer_data_inputs(id).at(0)).piece_shape();
        auto const& wp = ps.piece_shape();
        const double width = wp.dims.empty() ? 1.0 : static_cast<double>(wp.dims.back());
        upd = std::min(elems, static_cast<double>(ip.num_elements()) * width);
      }
      for (int d : ds)
        if (d < static_cast<int>(params_on.size())) params_on[d] += upd;
      if (ps.discard_copy_degree <= 1) continue;
      const bool gemm_w = wi == 0 && (node.label.op.type == OpType::LINEAR ||
                                      node.label.op.type == OpType::MULTIHEAD_ATTENTION);
      const double bytes = elems * ((cfg_.bf16_weight_grads && gemm_w) ? 2.0 : 4.0);
      const int c = ps.discard_copy_degree;
      if (cfg_.parameter_server) {
        // gradients of the c copies into the group leader, leader update,
        // weights back to the copies (barrier -> update -> final)
        const double in_bw = std::max(1, std::min(c - 1, spec.xgmi_links)) * spec.xgmi_link_bandwidth;
        const double gather = (c - 1) * bytes / in_bw + spec.collective_latency;
        int r = push(SimTask::REDUCE, id, node.label.name + ":ps_reduce" + std::to_string(wi), ds, gather, COMM_LANE);
        tasks[r].deps.push_back({k, 0.0});
        const int lead_n = std::max<int>(1, static_cast<int>(P.size()) / c);
        std::vector<int> leaders = devset(Placement(P.begin(), P.begin() + std::min<size_t>(P.size(), lead_n)));
        int u = push(SimTask::UPDATE, id, node.label.name + ":ps_update" + std::to_string(wi), leaders,
                     elems * cfg_.update_bytes_per_param / spec.hbm_bandwidth + spec.kernel_launch_overhead,
                     COMPUTE_LANE);
        tasks[u].deps.push_back({r, 0.0});
        const double bcast = (c - 1) * elems * 4.0 / in_bw + spec.collective_latency;
        int b = push(SimTask::BCAST, id, node.label.name + ":ps_bcast" + std::to_string(wi), ds, bcast, COMM_LANE);
        tasks[b].deps.push_back({u, 0.0});
        res.sync_time += gather + bcast;
        ps_final.push_back(b);
        for (int d : ds) sync_on[d].push_back(b);
        continue;
      }
      auto& bk = buckets[{ds, c}];
      bk.copy = c;
      bk.devs = ds;
      bk.bytes += bytes;
      bk.last_task = k;
      if (cfg_.overlap_grad_sync && bk.bytes >= cfg_.bucket_bytes) emit_allreduce(bk, k);
    }
  }
  for (auto& kv : buckets) emit_allreduce(kv.second, last_bwd >= 0 ? last_bwd : kv.second.last_task);
  // optimizer update per device, after its last backward and its syncs
  if (cfg_.include_update && !cfg_.parameter_server) {
    for (int d = 0; d < world; ++d) {
      if (params_on[d] <= 0) continue;
      const double run = params_on[d] * cfg_.update_bytes_per_param / spec.hbm_bandwidth + 2 * spec.kernel_launch_overhead;
      int k = push(SimTask::UPDATE, -1, "update", {d}, run, COMPUTE_LANE);
      res.update_time = std::max(res.update_time, run);
      if (last_bwd_on[d] >= 0) tasks[k].deps.push_back({last_bwd_on[d], 0.0});
      for (int s : sync_on[d]) tasks[k].deps.push_back({s, 0.0});
    }
  }

  // ---- list scheduling in creation order (= each rank's issue order)
  std::vector<double> comp(world + 64, 0.0), comm(world + 64, 0.0);
  std::map<int, double> link_free;
  std::map<std::pair<int, int>, double> pair_free;
  double end = 0, fwd_end = 0, bwd_end = 0;
  auto lane_of = [&](const Rec& r) -> std::vector<double>& { return r.lane == COMM_LANE ? comm : comp; };
  for (auto& r : tasks) {
    double ready = 0;
    for (auto const& d : r.deps) ready = std::max(ready, tasks[d.first].t.end_time + d.second);
    double start = ready;
    auto& lane = lane_of(r);
    for (int d : r.t.devices)
      if (d >= 0 && d < static_cast<int>(lane.size())) start = std::max(start, lane[d]);
    if (r.t.type == SimTask::XFER) {
      if (!r.t.links.empty()) {
        for (int l : r.t.links) start = std::max(start, link_free[l]);
      } else {
        start = std::max(start, pair_free[{r.t.src, r.t.dst}]);
      }
    }
    r.t.ready_time = ready;
    r.t.start_time = start;
    r.t.end_time = start + r.t.run_time;
    for (int d : r.t.devices)
      if (d >= 0 && d < static_cast<int>(lane.size())) lane[d] = r.t.end_time;
    if (r.t.type == SimTask::XFER) {
      for (int l : r.t.links) link_free[l] = r.t.end_time;
      if (r.t.links.empty()) pair_free[{r.t.src, r.t.dst}] = r.t.end_time;
    }
    end = std::max(end, r.t.end_time);
    const bool is_fwd = r.t.type == SimTask::FORWARD ||
                        (r.t.type == SimTask::COMM && r.t.name.size() > 4 &&
                         r.t.name.compare(r.t.name.size() - 4, 4, ":fwd") == 0);
    const bool is_bwd = r.t.type == SimTask::BACKWARD ||
                        (r.t.type == SimTask::COMM && r.t.name.size() > 4 &&
                         r.t.name.compare(r.t.name.size() - 4, 4, ":bwd") == 0);
    if (is_fwd) fwd_end = std::max(fwd_end, r.t.end_time);
    if (is_bwd) bwd_end = std::max(bwd_end, r.t.end_time);
  }
  // ---- memory per device
  // resident bytes add up; an op's transient workspace (measured allocator
  // peak) only while it runs, so each device adds its largest one
  std::vector<double> mem(world, 0.0), ws(world, 0.0);
  for (int id : order) {
    if (!active(id)) continue;
    for (int d : devset(place(id)))
      if (d >= 0 && d < world) {
        mem[d] += cost[id].memory;
        ws[d] = std::max(ws[d], cost[id].workspace);
      }
  }
  for (int d = 0; d < world; ++d) mem[d] += ws[d];
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
      for (auto const& d : r.deps) r.t.deps.push_back(d.first);
      res.tasks.push_back(r.t);
    }
  return res;
}

std::string Simulator::task_graph_dot(const SimResult& r) const {
  static const char* kind[] = {"FWD", "BWD", "COMM", "UPDATE", "ALLREDUCE", "XFER", "REDUCE", "BCAST", "BARRIER"};
  static const char* color[] = {"lightblue", "lightsalmon", "khaki", "palegreen", "plum", "gold", "orchid",
                                "orchid", "grey"};
  std::ostringstream os;
  os << "digraph taskgraph {\n  node [shape=box, style=filled];\n";
  for (size_t i = 0; i < r.tasks.size(); ++i) {
    auto const& t = r.tasks[i];
    os << "  t" << i << " [label=\"" << t.name << "\\n" << kind[t.type];
    if (t.type == SimTask::XFER) os << " " << t.src << "->" << t.dst << " " << t.bytes / 1e6 << " MB";
    else os << " dev[" << t.dev_start << "," << t.dev_start + t.dev_size << ")";
    os << "\\n" << t.run_time * 1e3 << " ms @ " << t.start_time * 1e3 << "\", fillcolor=" << color[t.type] << "];\n";
  }
  for (size_t i = 0; i < r.tasks.size(); ++i)
    for (int d : r.tasks[i].deps) os << "  t" << d << " -> t" << i << ";\n";
  os << "}\n";
  return os.str();
}

}  // namespace ff
