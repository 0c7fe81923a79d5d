// Liveness-based memory plan of a training step (see ff/memory_plan.h).
#include "ff/memory_plan.h"

#include <algorithm>
#include <cmath>
#include <set>

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

TensorShape node_output_piece(const ParallelComputationGraph& pcg, int n) {
  return pcg.g.node(n).outputs.at(0).shape.piece_shape();
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

  // executor fusions (MemoryPlanConfig::executor_fusions): nodes whose
  // outputs are never materialised, nodes whose gradient overwrites their
  // output, and per-node multipliers of the kept activation
  std::set<int> no_act, no_grad, keep_grad;
  // own_extra[n]: bytes (as a multiple of the output) n's backward reads
  // besides its output, alive until bwd(n) -- the pre-activation of a Linear
  // with an activation, attention's projections and output
  std::map<int, double> own_extra;
  if (cfg.executor_fusions) {
    auto type_of = [&](int n) { return pcg.g.node(n).label.op.type; };
    auto sole = [&](int n) -> int {
      auto it = consumers.find(n);
      return it != consumers.end() && it->second.size() == 1 ? it->second[0] : -1;
    };
    for (int n : order) {
      if (roles.at(n) != NodeRole::COMPUTE) continue;
      const auto& op = pcg.g.node(n).label.op;
      const OpType t = op.type;
      if (t == OpType::BATCHNORM && !(op.has("relu") && op.b("relu"))) {
        const int add = sole(n);
        if (add >= 0 && type_of(add) == OpType::EW_ADD && !no_act.count(add)) {
          const int relu = sole(add);
          if (relu >= 0 && type_of(relu) == OpType::RELU) {
            // neither output is stored; the fused backward does materialise the
            // masked gradient of the sum once (handed to the residual branch)
            no_act.insert(n);
            no_act.insert(add);
            no_grad.insert(n);
            keep_grad.insert(add);
          }
        }
      } else if (t == OpType::SOFTMAX && !consumers.count(n)) {
        no_act.insert(n);
        for (auto const& v : pcg.layer_data_inputs(n)) no_grad.insert(v.node);
      } else if (t == OpType::LINEAR) {
        const std::string a = op.has("activation") ? op.s("activation") : "none";
        if (!a.empty() && a != "none") own_extra[n] = 1.0;
      } else if (t == OpType::MULTIHEAD_ATTENTION) {
        auto ins = pcg.layer_data_inputs(n);
        if (ins.size() == 3) {
          const auto q = pcg.shape(ins[0]).piece_shape(), k = pcg.shape(ins[1]).piece_shape();
          const auto o = node_output_piece(pcg, n);
          const int64_t E = op.i("embed_dim"), H = std::max<int64_t>(1, op.i("num_heads"));
          const int64_t kd = op.i("kdim") > 0 ? op.i("kdim") : E / H, vd = op.i("vdim") > 0 ? op.i("vdim") : E / H;
          const double Sq = static_cast<double>(q.num_elements()) / std::max<int64_t>(1, q.dims.back());
          const double Sk = static_cast<double>(k.num_elements()) / std::max<int64_t>(1, k.dims.back());
          const double hd = static_cast<double>(H) / std::max(1, pcg.shape(ins[0]).discard_copy_degree);
          const double extra = hd * (Sq * kd + Sk * kd + Sk * vd + Sq * vd);
          const double out = static_cast<double>(o.num_elements());
          if (out > 0) own_extra[n] = extra / out;
        }
      }
    }
  }

  // which saved tensors the executor's backward reads (the op
  // implementations' saved tuples, flexflow_train_amd/ops/*.py): an output
  // nobody's backward reads leaves memory after its last forward reader
  // (runtime/executor.py drops it from the environment); unknown operators
  // are assumed to read both
  auto reads_own_output = [&](int n) {
    const auto& op = pcg.g.node(n).label.op;
    switch (op.type) {
      case OpType::LINEAR:
      case OpType::BATCHMATMUL:
      case OpType::EW_ADD:
      case OpType::EW_SUB:
      case OpType::EW_MUL:
      case OpType::EW_DIV:
      case OpType::MULTIHEAD_ATTENTION:
      case OpType::LAYERNORM:
      case OpType::POOL2D:
      case OpType::EMBEDDING:
      case OpType::CONCAT:
      case OpType::SPLIT:
      case OpType::DROPOUT:
      case OpType::RESHAPE:
      case OpType::FLAT:
      case OpType::TRANSPOSE:
      case OpType::REVERSE:
      case OpType::GELU:
      case OpType::IDENTITY:
        return false;
      case OpType::CONV2D:
        return op.has("activation") && op.s("activation") != "none" && !op.s("activation").empty();
      case OpType::BATCHNORM:
        return op.has("relu") && op.b("relu");
      default:
        return true;
    }
  };
  auto reads_inputs = [&](int c) {
    switch (pcg.g.node(c).label.op.type) {
      case OpType::EW_ADD:
      case OpType::EW_SUB:
      case OpType::CONCAT:
      case OpType::SPLIT:
      case OpType::DROPOUT:
      case OpType::RESHAPE:
      case OpType::FLAT:
      case OpType::TRANSPOSE:
      case OpType::REVERSE:
      case OpType::SOFTMAX:
      case OpType::RELU:
      case OpType::SIGMOID:
      case OpType::TANH:
      case OpType::POOL2D:
      case OpType::IDENTITY:
        return false;
      default:
        return roles.at(c) != NodeRole::WEIGHT_PATH;
    }
  };

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
    if (no_act.count(n) && !keep_grad.count(n)) continue;
    const bool store_act = !no_act.count(n);
    const double extra = own_extra.count(n) ? own_extra.at(n) : 0.0;
    // the output's last reader: n's own backward, a consumer's backward that
    // reads it, or (executor fusions, nobody's backward reads it) its last
    // forward consumer.  The loss-fused softmax's logits hold their gradient.
    int out_end = bwd(n);
    if (cfg.training && cfg.executor_fusions && role == NodeRole::COMPUTE && !reads_own_output(n) &&
        !no_grad.count(n)) {
      out_end = last_fwd;
      for (int c : consumers[n])
        if (reads_inputs(c)) out_end = std::max(out_end, bwd(c));
    }
    for (size_t o = 0; o < node.outputs.size(); ++o) {
      const auto& s = node.outputs[o].shape;
      const double bytes = cfg.act_elem_bytes > 0
                               ? static_cast<double>(s.piece_shape().num_elements()) * cfg.act_elem_bytes
                               : static_cast<double>(s.piece_shape().size_bytes());
      for (auto const& h : holders(place(n), total_pieces(s))) {
        if (h.first < 0 || h.first >= world) continue;
        MemBlock a;
        a.node = n;
        a.output = static_cast<int>(o);
        a.kind = 0;
        a.bytes = bytes * h.second * copies;
        a.start = fwd.at(n);
        // inputs fed to the graph are read by their consumers' backward
        // (weight gradients); every other activation until its last reader
        a.end = !cfg.training ? last_fwd : role == NodeRole::INPUT_PATH ? std::max(last_fwd, steps - 1 - fwd.at(n))
                                                                        : out_end;
        if (store_act) {
          plans[h.first].blocks.push_back(a);
          if (extra > 0) {
            MemBlock x = a;
            x.bytes = a.bytes * extra;
            x.end = cfg.training ? bwd(n) : last_fwd;
            plans[h.first].blocks.push_back(x);
          }
        }
        if (grad && !no_grad.count(n)) {
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
