// Pipeline-parallel candidates for the strategy search (see ff/pipeline.h).
#include "ff/pipeline.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <numeric>
#include <set>

namespace ff {

Json PipelinePlan::to_json(bool with_views) const {
  Json j = Json::object();
  j["stages"] = static_cast<int64_t>(stages);
  j["micro_batches"] = static_cast<int64_t>(micro_batches);
  j["stage_degree"] = static_cast<int64_t>(stage_degree);
  j["step_time"] = step_time;
  j["bubble_fraction"] = bubble_fraction;
  j["stage_time"] = Json(stage_time);
  j["stage_sync"] = Json(stage_sync);
  j["stage_update"] = Json(stage_update);
  j["stage_activation_bytes"] = Json(stage_activation_bytes);
  if (with_views) {
    Json so = Json::object();
    for (auto const& kv : stage_of) so[std::to_string(kv.first)] = static_cast<int64_t>(kv.second);
    j["stage_of"] = so;
  }
  return j;
}

double micro_batched_step_time(const SimResult& r, int m) {
  m = std::max(1, m);
  const double fb = std::max(0.0, r.backward_end);
  return m * fb + std::max(0.0, r.iteration_time - fb);
}

namespace {

// the smallest max-load split of `w` (in order) into at most k contiguous
// groups: binary search on the load, greedy feasibility; returns group ids
std::vector<int> linear_partition(const std::vector<double>& w, int k) {
  const double total = std::accumulate(w.begin(), w.end(), 0.0);
  double lo = w.empty() ? 0.0 : *std::max_element(w.begin(), w.end()), hi = std::max(total, lo);
  auto groups_for = [&](double cap, std::vector<int>* out) {
    int g = 0;
    double cur = 0;
    for (size_t i = 0; i < w.size(); ++i) {
      if (cur + w[i] > cap && cur > 0) {
        ++g;
        cur = 0;
      }
      cur += w[i];
      if (out) (*out)[i] = g;
    }
    return g + 1;
  };
  for (int it = 0; it < 60 && hi - lo > 1e-12 * std::max(1.0, hi); ++it) {
    const double mid = 0.5 * (lo + hi);
    if (groups_for(mid, nullptr) <= k) hi = mid;
    else lo = mid;
  }
  std::vector<int> out(w.size(), 0);
  groups_for(hi, &out);
  // exactly k non-empty stages when there are enough items: split the
  // largest groups' tails while fewer than k
  int used = out.empty() ? 0 : out.back() + 1;
  while (used < k && static_cast<int>(w.size()) >= k) {
    // find the group with the most items and split it in the middle
    std::map<int, std::vector<size_t>> members;
    for (size_t i = 0; i < out.size(); ++i) members[out[i]].push_back(i);
    int big = -1;
    size_t bsz = 0;
    for (auto const& kv : members)
      if (kv.second.size() > bsz) big = kv.first, bsz = kv.second.size();
    if (bsz < 2) break;
    const size_t cut = members[big][bsz / 2];
    for (size_t i = cut; i < out.size(); ++i) ++out[i];
    ++used;
  }
  return out;
}

}  // namespace

PipelinePlan price_pipeline(const ComputationGraph& cg, const CostModel& cm, int world, int stages, int m,
                            const SimConfig& sim) {
  if (stages < 1 || world % stages) throw FFError("pipeline: world must be a multiple of the stage count");
  PipelinePlan P;
  P.stages = stages;
  P.micro_batches = std::max(1, m);
  P.stage_degree = world / stages;
  P.pcg = data_parallel_pcg(cg, P.stage_degree);
  const auto& pcg = P.pcg;
  auto roles = classify_nodes(pcg);
  // data-path operators in topological order with their per-micro-batch cost
  std::vector<int> ops;
  std::vector<double> w;
  std::map<int, OpCost> cost;
  for (int n : pcg.g.topo_order()) {
    if (roles.at(n) == NodeRole::WEIGHT_PATH || roles.at(n) == NodeRole::INPUT_PATH) continue;
    OpCost c = pcg_node_cost(cm, pcg, n, P.stage_degree);
    cost[n] = c;
    ops.push_back(n);
    w.push_back(c.forward + c.backward);
  }
  if (static_cast<int>(ops.size()) < stages) throw FFError("pipeline: fewer operators than stages");
  auto part = linear_partition(w, stages);
  P.stage_time.assign(stages, 0.0);
  P.stage_sync.assign(stages, 0.0);
  P.stage_update.assign(stages, 0.0);
  P.stage_activation_bytes.assign(stages, 0.0);
  for (size_t i = 0; i < ops.size(); ++i) P.stage_of[ops[i]] = std::min(stages - 1, part[i]);
  // input-path nodes go with their first consumer's stage, weight-path nodes too
  std::map<int, std::vector<int>> users;
  for (int id : pcg.g.node_ids())
    for (auto const& v : pcg.g.node(id).inputs) users[v.node].push_back(id);
  std::function<int(int)> stage_of = [&](int id) -> int {
    auto it = P.stage_of.find(id);
    if (it != P.stage_of.end()) return it->second;
    int s = stages - 1;
    for (int u : users[id]) s = std::min(s, stage_of(u));
    P.stage_of[id] = s;
    return s;
  };
  for (int id : pcg.g.node_ids()) stage_of(id);
  auto block = [&](int s) { return block_placement(s * P.stage_degree, P.stage_degree); };
  for (auto const& kv : P.stage_of) P.views[kv.first] = block(kv.second);

  const auto& spec = cm.spec();
  for (int n : ops) {
    const int s = P.stage_of.at(n);
    const OpCost& c = cost.at(n);
    P.stage_time[s] += c.forward + c.backward;
    P.stage_sync[s] += c.sync;
    for (auto const& o : pcg.g.node(n).outputs) P.stage_activation_bytes[s] += o.shape.piece_shape().size_bytes();
    double params = 0;
    for (auto const& v : pcg.layer_weights(n)) params += static_cast<double>(pcg.shape(v).piece_shape().num_elements());
    if (sim.include_update) P.stage_update[s] += params * sim.update_bytes_per_param / spec.hbm_bandwidth;
    // boundary sends: a tensor consumed on a later stage moves there forward
    // (activation) and back (its gradient), once per micro-batch
    std::set<int> sent;
    for (int u : users[n]) {
      auto it = P.stage_of.find(u);
      if (it == P.stage_of.end() || it->second == s || sent.count(it->second)) continue;
      if (roles.at(u) == NodeRole::WEIGHT_PATH) continue;
      sent.insert(it->second);
      P.stage_time[s] += 2.0 * cm.movement_cost(pcg.g.node(n).outputs.at(0).shape, block(s), block(it->second));
    }
  }
  const double slot = *std::max_element(P.stage_time.begin(), P.stage_time.end());
  const int M = P.micro_batches;
  P.bubble_fraction = static_cast<double>(stages - 1) / (M + stages - 1);
  P.step_time = (M + stages - 1) * slot + *std::max_element(P.stage_sync.begin(), P.stage_sync.end()) +
                *std::max_element(P.stage_update.begin(), P.stage_update.end());
  return P;
}

MemoryPlanConfig pipeline_memory_config(const PipelinePlan& p, bool one_f_one_b) {
  MemoryPlanConfig c;
  const int m = std::max(1, p.micro_batches);
  for (auto const& kv : p.stage_of)
    c.live_copies[kv.first] = one_f_one_b ? std::min(m, std::max(1, p.stages - kv.second)) : m;
  return c;
}

std::vector<PipelinePlan> pipeline_candidates(const ComputationGraph& cg, const CostModel& cm, int world,
                                              int micro_batches, const SimConfig& sim) {
  std::vector<PipelinePlan> out;
  for (int s = 2; s <= world; ++s) {
    if (world % s) continue;
    try {
      out.push_back(price_pipeline(cg, cm, world, s, micro_batches, sim));
    } catch (const FFError&) {
    }
  }
  return out;
}

}  // namespace ff
