#include "ff/mapping.h"

#include <functional>
#include <limits>
#include <optional>
#include <set>

namespace ff {

static constexpr double kInf = std::numeric_limits<double>::infinity();

Json MachineMappingResult::to_json() const {
  Json j = Json::object();
  j["runtime"] = runtime;
  j["feasible"] = feasible;
  Json v = Json::object();
  for (auto const& kv : views) v[std::to_string(kv.first)] = Json(std::vector<int64_t>{kv.second.start, kv.second.size});
  j["views"] = v;
  return j;
}

MachineMapper::MachineMapper(const ParallelComputationGraph& pcg, MachineMappingContext ctx)
    : pcg_(pcg), ctx_(ctx) {
  if (!ctx_.cost) throw FFError("MachineMapper: no cost model");
  roles_ = classify_nodes(pcg_);
  tree_ = get_relaxed_sp_decomposition(data_path_digraph(pcg_));
}

MachineMappingResult MachineMapper::leaf(int node, const DeviceBlock& res) {
  MachineMappingResult r;
  auto role = roles_.at(node);
  auto const& n = pcg_.g.node(node);
  if (n.outputs.empty()) {
    r.views[node] = res;
    return r;
  }
  int T = n.outputs[0].shape.total_parallel_degree();
  // largest aligned block inside `res` whose size is a multiple of T
  DeviceBlock best{res.start, 0};
  if (res.size % T == 0) best.size = res.size;
  else if (ctx_.allow_sub_blocks) {
    for (int s = res.size; s >= T; --s)
      if (s % T == 0) {
        best.size = s;
        break;
      }
  }
  if (best.size == 0) {
    r.feasible = false;
    r.runtime = kInf;
    return r;
  }
  r.views[node] = best;
  if (role == NodeRole::COMPUTE || role == NodeRole::PARALLEL) {
    OpCost c = pcg_node_cost(*ctx_.cost, pcg_, node, best.size);
    r.runtime = c.forward + c.backward + (ctx_.include_sync ? c.sync : 0.0);
  }
  return r;
}

double MachineMapper::movement(const std::vector<int>& left_leaves, const std::vector<int>& right_leaves,
                               const MachineMappingResult& l, const MachineMappingResult& r) {
  std::set<int> left(left_leaves.begin(), left_leaves.end());
  double t = 0;
  for (int n : right_leaves) {
    auto bn = r.views.at(n);
    for (auto const& v : pcg_.g.node(n).inputs) {
      if (!left.count(v.node)) continue;
      auto bp = l.views.at(v.node);
      if (bp == bn) continue;
      t += 2.0 * ctx_.cost->movement_cost(pcg_.shape(v), bp, bn);  // activation forward + gradient backward
    }
  }
  return t;
}

static MachineMappingResult merge(const MachineMappingResult& a, const MachineMappingResult& b, double runtime) {
  MachineMappingResult r;
  r.runtime = runtime;
  r.feasible = a.feasible && b.feasible;
  r.views = a.views;
  r.views.insert(b.views.begin(), b.views.end());
  return r;
}

MachineMappingResult MachineMapper::solve_node(int idx, const DeviceBlock& res) {
  auto key = std::make_pair(idx, res);
  auto it = cache_.find(key);
  if (it != cache_.end()) return it->second;
  auto const& e = tree_.e.at(idx);
  MachineMappingResult out;
  if (e.kind == SPTree::LEAF) {
    out = leaf(e.node, res);
  } else {
    auto l = solve_node(e.left, res);
    auto r = solve_node(e.right, res);
    if (!leaves_of_.count(e.left)) leaves_of_[e.left] = tree_.leaves(e.left);
    if (!leaves_of_.count(e.right)) leaves_of_[e.right] = tree_.leaves(e.right);
    if (e.kind == SPTree::SERIES) {
      double comm = (l.feasible && r.feasible) ? movement(leaves_of_[e.left], leaves_of_[e.right], l, r) : 0.0;
      out = merge(l, r, l.runtime + comm + r.runtime);
    } else {
      out = merge(l, r, l.runtime + r.runtime);  // both branches serially on the full resource
      for (auto const& sp : get_resource_splits(res)) {
        auto a = solve_node(e.left, sp.first);
        if (!a.feasible) continue;
        auto b = solve_node(e.right, sp.second);
        if (!b.feasible) continue;
        double t = std::max(a.runtime, b.runtime);
        if (t < out.runtime) out = merge(a, b, t);
      }
    }
    if (!out.feasible) out.runtime = kInf;
  }
  cache_[key] = out;
  return out;
}

MachineMappingResult MachineMapper::solve(const DeviceBlock& resources) {
  if (tree_.root < 0) return MachineMappingResult{};
  auto r = solve_node(tree_.root, resources);
  // weight-path nodes follow their (first) data-path consumer
  std::map<int, std::vector<int>> users;
  for (int id : pcg_.g.node_ids())
    for (auto const& v : pcg_.g.node(id).inputs) users[v.node].push_back(id);
  std::function<std::optional<DeviceBlock>(int)> consumer_block = [&](int id) -> std::optional<DeviceBlock> {
    for (int u : users[id]) {
      auto jt = r.views.find(u);
      if (jt != r.views.end() && roles_.at(u) != NodeRole::WEIGHT_PATH) return jt->second;
      auto b = consumer_block(u);
      if (b) return b;
    }
    return std::nullopt;
  };
  for (int id : pcg_.g.node_ids())
    if (roles_.at(id) == NodeRole::WEIGHT_PATH) {
      auto b = consumer_block(id);
      r.views[id] = b ? *b : resources;
    }
  return r;
}

MachineMappingResult get_optimal_machine_mapping(const ParallelComputationGraph& pcg, const CostModel& cm,
                                                 int world) {
  MachineMappingContext ctx;
  ctx.cost = &cm;
  MachineMapper m(pcg, ctx);
  return m.solve(DeviceBlock{0, world});
}

}  // namespace ff
