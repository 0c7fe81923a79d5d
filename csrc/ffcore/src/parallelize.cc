#include "ff/parallelize.h"

#include <algorithm>
#include <sstream>
#include <tuple>

namespace ff {

std::string mp_kind_to_string(MPKind k) {
  switch (k) {
    case MPKind::NONE: return "none";
    case MPKind::COLUMN: return "column";
    case MPKind::ROW: return "row";
    case MPKind::HEADS: return "heads";
    case MPKind::EXPERTS: return "experts";
  }
  return "none";
}

MPKind mp_kind_from_string(const std::string& s) {
  if (s == "column") return MPKind::COLUMN;
  if (s == "row") return MPKind::ROW;
  if (s == "heads") return MPKind::HEADS;
  if (s == "experts") return MPKind::EXPERTS;
  if (s == "none" || s.empty()) return MPKind::NONE;
  throw FFError("unknown model-parallel kind '" + s + "'");
}

bool LayerConfig::operator<(const LayerConfig& o) const {
  return std::make_tuple(batch, seq, model, static_cast<int>(kind)) <
         std::make_tuple(o.batch, o.seq, o.model, static_cast<int>(o.kind));
}

std::string LayerConfig::str() const {
  std::ostringstream os;
  os << "b" << batch;
  if (seq > 1) os << ".s" << seq;
  if (kind != MPKind::NONE) os << "." << mp_kind_to_string(kind) << model;
  return os.str();
}

Json LayerConfig::to_json() const {
  Json j = Json::object();
  j["batch"] = batch;
  j["seq"] = seq;
  j["model"] = model;
  j["kind"] = mp_kind_to_string(kind);
  return j;
}

LayerConfig LayerConfig::from_json(const Json& j) {
  LayerConfig c;
  c.batch = static_cast<int>(j.at("batch").as_int());
  if (j.contains("seq")) c.seq = static_cast<int>(j.at("seq").as_int());
  if (j.contains("model")) c.model = static_cast<int>(j.at("model").as_int());
  if (j.contains("kind")) c.kind = mp_kind_from_string(j.at("kind").as_string());
  return c;
}

namespace {

std::vector<int> divisors(int n) {
  std::vector<int> r;
  for (int d = 1; d <= n; ++d)
    if (n % d == 0) r.push_back(d);
  return r;
}

bool is_mp_capable(const OpAttrs& op, MPKind k) {
  switch (op.type) {
    case OpType::LINEAR:
      if (k == MPKind::COLUMN) return true;
      if (k == MPKind::ROW) return activation_from_string(op.s("activation")) == Activation::NONE;
      return false;
    case OpType::MULTIHEAD_ATTENTION: return k == MPKind::HEADS;
    case OpType::EXPERTS: return k == MPKind::EXPERTS;
    case OpType::EMBEDDING: return k == MPKind::COLUMN && op.s("aggr") == "none";
    // conv channel parallelism (op-attrs conv_2d.cc:85-142): COLUMN = output
    // channels (weight sharded on K), ROW = input channels (partial sums)
    case OpType::CONV2D:
      if (op.i("groups") != 1) return false;
      if (k == MPKind::COLUMN) return true;
      if (k == MPKind::ROW) return activation_from_string(op.s("activation")) == Activation::NONE;
      return false;
    default: return false;
  }
}

// The attribute dim the `seq` degree shards: the sequence (dim 1) of a
// [batch, seq, ...] activation, H (dim 2) of an NCHW image.
int attribute_dim(const TensorShape& s) { return s.num_dims() == 4 ? 2 : 1; }

// Degrees for a data input of rank r / dims under (batch, seq), with the
// leading-dim sizes of input 0 used to detect broadcast operands.
ParallelTensorShape batch_seq_shape(const TensorShape& s, const TensorShape& ref, int b, int q) {
  std::vector<int> deg(s.num_dims(), 1);
  if (s.num_dims() >= 1 && b > 1 && s.num_dims() == ref.num_dims() && s.dims[0] == ref.dims[0] &&
      s.dims[0] % b == 0)
    deg[0] = b;
  const int ad = attribute_dim(s);
  if (s.num_dims() >= 3 && q > 1 && s.num_dims() == ref.num_dims() && s.dims[ad] == ref.dims[ad] &&
      s.dims[ad] % q == 0)
    deg[ad] = q;
  return lift_to_parallel_with_degrees(s, 1, 1, deg);
}

}  // namespace

OpAttrs configured_op(const OpAttrs& op, const LayerConfig& cfg) {
  if (op.type == OpType::EXPERTS && cfg.kind == MPKind::EXPERTS && op.s("expert_parallel_mode") == "alltoall") {
    OpAttrs o = op;
    o.set("expert_degree", static_cast<int64_t>(cfg.model));
    return o;
  }
  return op;
}

std::optional<std::vector<ParallelTensorShape>> required_input_shapes(const ComputationGraph& cg, int node,
                                                                      const LayerConfig& cfg) {
  auto const& n = cg.g.node(node);
  const OpAttrs op = configured_op(n.label.op, cfg);
  auto data = cg.layer_data_inputs(node);
  if (data.empty()) return std::vector<ParallelTensorShape>{};
  std::vector<TensorShape> ss;
  for (auto const& v : data) ss.push_back(cg.shape(v));
  const TensorShape& ref = ss[0];
  std::vector<ParallelTensorShape> ps;
  for (auto const& s : ss) {
    auto p = batch_seq_shape(s, ref, cfg.batch, cfg.seq);
    ps.push_back(p);
  }
  // every requested degree must actually apply to input 0
  if (cfg.batch > 1 && (ref.num_dims() < 1 || ps[0].dim(0).degree != cfg.batch)) return std::nullopt;
  if (cfg.seq > 1 && (ref.num_dims() < 3 || ps[0].dim(attribute_dim(ref)).degree != cfg.seq)) return std::nullopt;
  if (cfg.kind != MPKind::NONE || cfg.model > 1) {
    if (cfg.kind == MPKind::NONE || cfg.model <= 1 || !is_mp_capable(op, cfg.kind)) return std::nullopt;
    switch (cfg.kind) {
      case MPKind::COLUMN: {
        int64_t oc = op.i("out_channels");
        if (oc % cfg.model) return std::nullopt;
        ps[0].discard_copy_degree = cfg.model;
        break;
      }
      case MPKind::ROW: {
        // the reduction (input-feature) dim: channels (dim 1) for a conv, the last dim otherwise
        const int rd = op.type == OpType::CONV2D ? 1 : ref.num_dims() - 1;
        if (ref.dims[rd] % cfg.model) return std::nullopt;
        ps[0].shard_dims[rd].degree = cfg.model;
        break;
      }
      case MPKind::HEADS: {
        if (op.i("num_heads") % cfg.model) return std::nullopt;
        for (auto& p : ps) p.discard_copy_degree = cfg.model;
        break;
      }
      case MPKind::EXPERTS: {
        if (op.i("num_experts") % cfg.model) return std::nullopt;
        if (op.s("expert_parallel_mode") == "alltoall") {
          // tokens spread over batch x expert ranks, dispatched in the op
          const int64_t B = ref.dims[0];
          if (B % (static_cast<int64_t>(cfg.batch) * cfg.model)) return std::nullopt;
          for (auto& p : ps) p.shard_dims[0].degree = cfg.batch * cfg.model;
        } else {
          for (auto& p : ps) p.discard_copy_degree = cfg.model;
        }
        break;
      }
      default: return std::nullopt;
    }
  }
  for (auto const& p : ps)
    if (!p.is_valid()) return std::nullopt;
  try {
    if (!is_valid_parallelization(op, ps)) return std::nullopt;
    auto outs = infer_parallel_output_shapes(op, ps);
    for (auto const& o : outs)
      if (!o.is_valid()) return std::nullopt;
    auto ws = infer_parallel_weight_shapes(op, ps);
    for (auto const& w : ws)
      if (!w.is_valid()) return std::nullopt;
  } catch (const FFError&) {
    return std::nullopt;
  }
  return ps;
}

std::vector<LayerConfig> candidate_configs(const ComputationGraph& cg, int node, int world,
                                           const SearchSpaceOptions& opt) {
  auto const& op = cg.g.node(node).label.op;
  std::vector<LayerConfig> out;
  if (op.type == OpType::WEIGHT) return {LayerConfig{}};
  std::vector<MPKind> kinds{MPKind::NONE};
  if (opt.enable_parameter_parallel)
    for (MPKind k : {MPKind::COLUMN, MPKind::ROW, MPKind::HEADS, MPKind::EXPERTS})
      if (is_mp_capable(op, k)) kinds.push_back(k);
  for (int b : divisors(world))
    for (int q : divisors(world / b)) {
      if (q > 1 && !opt.enable_attribute_parallel) continue;
      for (MPKind k : kinds)
        for (int m : divisors(world / (b * q))) {
          if ((k == MPKind::NONE) != (m == 1)) continue;
          if (m > opt.max_model_degree) continue;
          LayerConfig c{b, q, m, k};
          if (!opt.allow_partial_world && c.total() != world) continue;
          if (op.type == OpType::INPUT) {
            auto const& s = cg.shape({node, 0});
            if (c.kind != MPKind::NONE || c.seq > 1) continue;
            if (b > 1 && (s.num_dims() < 1 || s.dims[0] % b)) continue;
            out.push_back(c);
            continue;
          }
          if (required_input_shapes(cg, node, c)) out.push_back(c);
        }
    }
  if (out.empty()) out.push_back(LayerConfig{});  // fully replicated always works
  return out;
}

StrategyConfig data_parallel_strategy(const ComputationGraph& cg, int world) {
  StrategyConfig s;
  for (int id : cg.g.topo_order()) {
    auto const& op = cg.g.node(id).label.op;
    if (op.type == OpType::WEIGHT) continue;
    LayerConfig c{world, 1, 1, MPKind::NONE};
    bool ok = false;
    if (op.type == OpType::INPUT) {
      auto const& sh = cg.shape({id, 0});
      ok = sh.num_dims() >= 1 && sh.dims[0] % world == 0;
    } else {
      ok = required_input_shapes(cg, id, c).has_value();
    }
    s[id] = ok ? c : LayerConfig{};
  }
  return s;
}

ValueRef convert_parallel_shape(ParallelComputationGraph& pcg, ValueRef v, const ParallelTensorShape& target,
                                int* num_ops) {
  auto cnt = [&]() {
    if (num_ops) ++*num_ops;
  };
  ParallelTensorShape s = pcg.shape(v);
  if (s.num_dims() != target.num_dims()) throw FFError("convert_parallel_shape: rank mismatch");
  if (s.sum_degree != target.sum_degree) {
    if (target.sum_degree != 1) throw FFError("convert_parallel_shape: cannot create partial sums");
    v = pcg.parallel_reduce(v, s.sum_degree);
    cnt();
    s = pcg.shape(v);
  }
  if (s.discard_copy_degree > target.discard_copy_degree)
    throw FFError("convert_parallel_shape: cannot drop replicas (" + s.str() + " -> " + target.str() + ")");
  for (int d = 0; d < s.num_dims(); ++d) {
    int a = s.shard_dims[d].degree, b = target.shard_dims[d].degree;
    if (a > b) {
      int f = (a % b == 0) ? a / b : a;
      v = pcg.parallel_combine(v, d, f);
      cnt();
    }
  }
  s = pcg.shape(v);
  for (int d = 0; d < s.num_dims(); ++d) {
    int a = s.shard_dims[d].degree, b = target.shard_dims[d].degree;
    if (a < b) {
      if (b % a) throw FFError("convert_parallel_shape: incompatible degrees");
      v = pcg.parallel_partition(v, d, b / a);
      cnt();
    }
  }
  s = pcg.shape(v);
  if (s.discard_copy_degree < target.discard_copy_degree) {
    if (target.discard_copy_degree % s.discard_copy_degree) throw FFError("convert_parallel_shape: replica degree");
    v = pcg.parallel_replicate(v, target.discard_copy_degree / s.discard_copy_degree);
    cnt();
  }
  if (pcg.shape(v) != target)
    throw FFError("convert_parallel_shape: produced " + pcg.shape(v).str() + " wanted " + target.str());
  return v;
}

Lowering lower_strategy(const ComputationGraph& cg, const StrategyConfig& cfg, int world) {
  Lowering L;
  auto& p = L.pcg;
  std::map<ValueRef, ValueRef> vm;
  std::map<std::pair<ValueRef, std::string>, ValueRef> conv_cache;
  auto get_cfg = [&](int id) {
    auto it = cfg.find(id);
    return it == cfg.end() ? LayerConfig{} : it->second;
  };
  auto convert = [&](ValueRef v, const ParallelTensorShape& t) {
    if (p.shape(v) == t) return v;
    auto key = std::make_pair(v, t.str());
    auto it = conv_cache.find(key);
    if (it != conv_cache.end()) return it->second;
    ValueRef r = convert_parallel_shape(p, v, t, &L.num_parallel_ops);
    conv_cache[key] = r;
    return r;
  };
  for (int id : cg.g.topo_order()) {
    auto const& n = cg.g.node(id);
    auto t = n.label.op.type;
    if (t == OpType::WEIGHT) continue;
    LayerConfig c = get_cfg(id);
    if (c.total() > world) throw FFError("layer " + n.label.name + ": config " + c.str() + " exceeds world");
    if (t == OpType::INPUT) {
      auto const& s = n.outputs[0].shape;
      ValueRef v = p.add_input(lift_to_parallel(s), n.outputs[0].create_grad, n.label.name);
      L.cg_to_pcg[id] = v.node;
      // constant inputs (no sample dimension) stay whole on every rank
      const bool replicated = n.label.op.has("replicated") && n.label.op.b("replicated");
      if (c.batch > 1 && !replicated) {
        if (s.num_dims() < 1 || s.dims[0] % c.batch) throw FFError("input " + n.label.name + ": batch degree");
        v = p.parallel_partition(v, 0, c.batch);
        ++L.num_parallel_ops;
      }
      vm[{id, 0}] = v;
      continue;
    }
    auto req = required_input_shapes(cg, id, c);
    if (!req) throw FFError("layer " + n.label.name + ": config " + c.str() + " is not valid for this op");
    auto data = cg.layer_data_inputs(id);
    auto wts = cg.layer_weights(id);
    std::vector<ValueRef> din;
    for (size_t i = 0; i < data.size(); ++i) din.push_back(convert(vm.at(data[i]), (*req)[i]));
    std::vector<ParallelTensorShape> ps;
    for (auto const& v : din) ps.push_back(p.shape(v));
    const OpAttrs op = configured_op(n.label.op, c);
    auto wshapes = infer_parallel_weight_shapes(op, ps);
    std::vector<ValueRef> all = din;
    for (size_t i = 0; i < wts.size(); ++i) {
      auto const& wn = cg.g.node(wts[i].node);
      all.push_back(p.add_weight(wn.outputs[0].shape, wshapes[i], wn.outputs[0].initializer,
                                 wn.outputs[0].create_grad, wn.label.name));
    }
    auto outs = p.add_layer(op, all, n.label.name);
    L.cg_to_pcg[id] = outs.empty() ? -1 : outs[0].node;
    for (size_t i = 0; i < outs.size(); ++i) vm[{id, static_cast<int>(i)}] = outs[i];
  }
  // sinks: resolve pending partial sums
  for (int id : cg.g.topo_order()) {
    auto t = cg.g.node(id).label.op.type;
    if (t == OpType::WEIGHT || t == OpType::INPUT) continue;
    for (size_t i = 0; i < cg.g.node(id).outputs.size(); ++i) {
      ValueRef cv{id, static_cast<int>(i)};
      if (!cg.g.uses(cv).empty()) continue;
      ValueRef v = vm.at(cv);
      auto s = p.shape(v);
      if (s.sum_degree > 1) {
        p.parallel_reduce(v, s.sum_degree);
        ++L.num_parallel_ops;
      }
    }
  }
  return L;
}

Json strategy_to_json(const ComputationGraph& cg, const StrategyConfig& s) {
  Json j = Json::object();
  for (auto const& kv : s) {
    auto const& nm = cg.g.node(kv.first).label.name;
    j[nm.empty() ? std::to_string(kv.first) : nm] = kv.second.to_json();
  }
  return j;
}

StrategyConfig strategy_from_json(const ComputationGraph& cg, const Json& j) {
  StrategyConfig s;
  for (int id : cg.g.node_ids()) {
    auto const& nm = cg.g.node(id).label.name;
    std::string key = nm.empty() ? std::to_string(id) : nm;
    if (j.contains(key)) s[id] = LayerConfig::from_json(j.at(key));
  }
  return s;
}

}  // namespace ff
