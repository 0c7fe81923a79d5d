// Liveness-based memory plan of a training step (see ff/memory_plan.h).
#include "ff/memory_plan.h"

#include <algorithm>
#include <cmath>

#include "ff/simulator.h"

namespace ff {

Json MemoryPlan::to_json(bool with_blocks) const {
  Json j = Json::object();
  j["device"] = static_cast<int64_t>(device);
  j["steps"] = static_cast<int64_t>(steps);
  j["weight_bytes"] = weight_bytes;
  j["peak_live_bytes"] = peak_live_bytes;
  j["arena_bytes"] = arena_bytes;
  j["naive_bytes"] = naive_bytes;
  j["num_blocks"] = static_cast<int64_t>(blocks.size());
  if (with_blocks) {
    Json a = Json::array();
    for (auto const& b : blocks) {
      Json e = Json::object();
      e["node"] = static_cast<int64_t>(b.node);
      e["output"] = static_cast<int64_t>(b.output);
      e["kind"] = static_cast<int64_t>(b.kind);
      e["bytes"] = b.bytes;
      e["start"] = static_cast<int64_t>(b.start);
      e["end"] = static_cast<int64_t>(b.end);
      e["offset"] = b.offset;
      a.push_back(e);
    }
    j["blocks"] = a;
  }
  return j;
}

namespace {

// devices holding pieces of a tensor with `pieces` pieces on placement `p`,
// and how many pieces each holds
std::vector<std::pair<int, double>> holders(const Placement& p, int pieces) {
  std::vector<int> d = p;
  std::sort(d.begin(), d.end());
  d.erase(std::unique(d.begin(), d.end()), d.end());
  std::vector<std::pair<int, double>> r;
  if (d.empty()) return r;
  const double per = std::max(1.0, static_cast<double>(pieces) / static_cast<double>(d.size()));
  for (int x : d) r.push_back({x, per});
  return r;
}

int total_pieces(const ParallelTensorShape& s) {
  int n = s.sum_degree * s.discard_copy_degree;
  for (int i = 0; i < s.num_dims(); ++i) n *= s.dim(i).degree;
  return std::max(1, n);
}

void pack(MemoryPlan& m, double align) {
  // peak of the live sum: sweep over steps
  std::vector<double> live(static_cast<size_t>(std::max(1, m.steps)) + 1, 0.0);
  for (auto const& b : m.blocks) {
    for (int t = b.start; t <= b.end && t < static_cast<int>(live.size()); ++t) live[t] += b.bytes;
    m.naive_bytes += b.bytes;
  }
  m.peak_live_bytes = live.empty() ? 0.0 : *std::max_element(live.begin(), live.end());
  // first fit decreasing: biggest blocks first, lowest offset free of every
  // placed block that is alive at the same time
  std::vector<size_t> idx(m.blocks.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return m.blocks[a].bytes > m.blocks[b].bytes; });
  std::vector<size_t> placed;
  double arena = 0;
  for (size_t i : idx) {
    MemBlock& b = m.blocks[i];
    const double sz = std::ceil(b.bytes / align) * align;
    std::vector<std::pair<double, double>> busy;   // [lo, hi) of time-overlapping placed blocks
    for (size_t j : placed) {
      const MemBlock& o = m.blocks[j];
      if (o.start <= b.end && b.start <= o.end)
        busy.push_back({o.offset, o.offset + std::ceil(o.bytes / align) * align});
    }
    std::sort(busy.begin(), busy.end());
    double off = 0;
    for (auto const& iv : busy) {
      if (off + sz <= iv.first) break;
      off = std::max(off, iv.second);
    }
    b.offset = off;
    arena = std::max(arena, off + sz);
    placed.push_back(i);
  }
  m.arena_bytes = arena;
}

}  // namespace

std::vector<MemoryPlan> plan_memory(const ParallelComputationGraph& pcg, const std::map<int, Placement>& views,
                                    int world, const MemoryPlanConfig& cfg) {
  world = std::max(1, world);
  std::vector<MemoryPlan> plans(world);
  for (int d = 0; d < world; ++d) plans[d].device = d;
  const auto roles = classify_nodes(pcg);
  const auto order = pcg.g.topo_order();
  const int N = static_cast<int>(order.size());
  const int steps = cfg.training ? 2 * N : N;
  std::map<int, int> fwd;
  for (int i = 0; i < N; ++i) fwd[order[i]] = i;
  auto bwd = [&](int n) { return 2 * N - 1 - fwd.at(n); };
  const Placement all = block_placement(0, world);
  auto place = [&](int n) -> const Placement& {
    auto it = views.find(n);
    return it == views.end() ? all : it->second;
  };
  std::map<int, std::vector<int>> consumers;
  for (int id : order)
    for (auto const& v : pcg.g.node(id).inputs) consumers[v.node].push_back(id);

  for (auto& p : plans) p.steps = steps;
  for (int n : order) {
    const auto& node = pcg.g.node(n);
    const NodeRole role = roles.at(n);
    if (role == NodeRole::WEIGHT_PATH) {
      // the weight itself (the WEIGHT node's outputs); its parallel ops
      // reshape what the consumers see -- count the pieces where they land
      bool feeds_op = false;
      for (int c : consumers[n]) feeds_op = feeds_op || roles.at(c) != NodeRole::WEIGHT_PATH;
      if (!feeds_op) continue;
      for (size_t o = 0; o < node.outputs.size(); ++o) {
        const auto& s = node.outputs[o].shape;
        const double bytes = static_cast<double>(s.piece_shape().num_elements()) * cfg.weight_bytes_per_param;
        for (auto const& h : holders(place(n), total_pieces(s))) {
          if (h.first < 0 || h.first >= world) continue;
          MemBlock b;
          b.node = n;
          b.output = static_cast<int>(o);
          b.kind = 2;
          b.bytes = bytes * h.second;
          b.start = 0;
          b.end = steps - 1;
          plans[h.first].blocks.push_back(b);
          plans[h.first].weight_bytes += b.bytes;
        }
      }
      continue;
    }
    int last_fwd = fwd.at(n), first_bwd = steps - 1;
    bool has_consumer = false;
    for (int c : consumers[n]) {
      has_consumer = true;
      last_fwd = std::max(last_fwd, fwd.at(c));
      if (cfg.training) first_bwd = std::min(first_bwd, bwd(c));
    }
    const bool grad = cfg.training && role != NodeRole::INPUT_PATH && has_consumer;
    auto lc = cfg.live_copies.find(n);
    const double copies = lc == cfg.live_copies.end() ? 1.0 : std::max(1.0, lc->second);
    for (size_t o = 0; o < node.outputs.size(); ++o) {
      const auto& s = node.outputs[o].shape;
      const double bytes = static_cast<double>(s.piece_shape().size_bytes());
      for (auto const& h : holders(place(n), total_pieces(s))) {
        if (h.first < 0 || h.first >= world) continue;
        MemBlock a;
        a.node = n;
        a.output = static_cast<int>(o);
        a.kind = 0;
        a.bytes = bytes * h.second * copies;
        a.start = fwd.at(n);
        // inputs fed to the graph are read by their consumers' backward
        // (weight gradients); every other activation until its producer's
        a.end = !cfg.training ? last_fwd : role == NodeRole::INPUT_PATH ? std::max(last_fwd, steps - 1 - fwd.at(n))
                                                                        : bwd(n);
        plans[h.first].blocks.push_back(a);
        if (grad) {
          MemBlock g = a;
          g.kind = 1;
          g.bytes = bytes * h.second;   // one micro-batch's gradient at a time
          g.start = first_bwd;
          g.end = bwd(n);
          plans[h.first].blocks.push_back(g);
        }
      }
    }
  }
  for (auto& p : plans) pack(p, cfg.align);
  return plans;
}

}  // namespace ff
