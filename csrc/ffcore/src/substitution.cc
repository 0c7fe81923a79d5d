#include "ff/substitution.h"

#include <algorithm>
#include <functional>
#include <map>
#include <sstream>

namespace ff {

// ---------------------------------------------------------------------------
// patterns
bool OperatorPattern::satisfied_by(const OpAttrs& op) const {
  if (type && op.type != *type) return false;
  for (auto const& c : attrs) {
    auto it = op.attrs.find(c.key);
    if (it == op.attrs.end()) return false;
    if (c.kind == AttrConstraint::EQUAL) {
      if (it->second != c.value) return false;
    } else {
      if (!std::holds_alternative<int64_t>(it->second) || !std::holds_alternative<int64_t>(c.value)) return false;
      int64_t d = std::get<int64_t>(c.value);
      if (d == 0 || std::get<int64_t>(it->second) % d != 0) return false;
    }
  }
  return true;
}

int PCGPattern::add_node(OperatorPattern p, std::vector<PatternValue> ins) {
  for (auto const& v : ins) {
    if (v.is_input()) num_inputs = std::max(num_inputs, v.input_index() + 1);
    else if (v.node >= static_cast<int>(nodes.size())) throw FFError("pattern: forward reference");
  }
  p.num_data_inputs = static_cast<int>(ins.size());
  nodes.push_back(std::move(p));
  inputs.push_back(std::move(ins));
  return static_cast<int>(nodes.size()) - 1;
}

static Json pv_json(const PatternValue& v) { return Json(std::vector<int64_t>{v.node, v.idx}); }

Json Substitution::to_json() const {
  Json j = Json::object();
  j["name"] = name;
  Json pn = Json::array();
  for (size_t i = 0; i < pattern.nodes.size(); ++i) {
    Json n = Json::object();
    n["type"] = pattern.nodes[i].type ? to_string(*pattern.nodes[i].type) : "*";
    Json c = Json::object();
    for (auto const& a : pattern.nodes[i].attrs) c[a.key] = attr_to_json(a.value);
    n["attrs"] = c;
    Json ins = Json::array();
    for (auto const& v : pattern.inputs[i]) ins.push_back(pv_json(v));
    n["inputs"] = ins;
    pn.push_back(n);
  }
  j["pattern"] = pn;
  Json po = Json::array();
  for (auto const& v : pattern.outputs) po.push_back(pv_json(v));
  j["pattern_outputs"] = po;
  Json on = Json::array();
  for (auto const& o : out_nodes) {
    Json n = Json::object();
    n["type"] = o.copy_from >= 0 ? "copy_of_" + std::to_string(o.copy_from) : to_string(o.type);
    Json a = Json::object();
    for (auto const& x : o.assign)
      a[x.key] = x.copy ? Json("copy:" + std::to_string(x.from_node) + "." + x.from_key) : attr_to_json(x.value);
    n["assign"] = a;
    Json ins = Json::array();
    for (auto const& v : o.inputs) ins.push_back(pv_json(v));
    n["inputs"] = ins;
    on.push_back(n);
  }
  j["output_graph"] = on;
  Json om = Json::array();
  for (auto const& v : output_mapping) om.push_back(pv_json(v));
  j["output_mapping"] = om;
  return j;
}

// ---------------------------------------------------------------------------
// matching
std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  size_t max_matches) {
  std::vector<PCGPatternMatch> out;
  const int np = static_cast<int>(p.nodes.size());
  if (np == 0) return out;
  // candidate pools (data-path nodes only)
  std::map<int, std::vector<std::pair<int, int>>> users;  // node -> (user, slot); per output idx encoded below
  std::map<ValueRef, std::vector<std::pair<int, int>>> vusers;
  std::vector<int> data_nodes;
  std::map<int, bool> weight_path;
  for (int id : pcg.g.topo_order()) {
    weight_path[id] = pcg.is_weight_path(id);
    auto const& n = pcg.g.node(id);
    if (!weight_path[id] && n.label.op.type != OpType::INPUT) data_nodes.push_back(id);
    for (size_t s = 0; s < n.inputs.size(); ++s) vusers[n.inputs[s]].push_back({id, static_cast<int>(s)});
  }
  // pattern adjacency and order (BFS from the most constrained node)
  std::vector<std::vector<std::pair<int, int>>> pusers(np);  // pattern node -> (user pnode, slot)
  for (int i = 0; i < np; ++i)
    for (size_t s = 0; s < p.inputs[i].size(); ++s)
      if (!p.inputs[i][s].is_input()) pusers[p.inputs[i][s].node].push_back({i, static_cast<int>(s)});
  int anchor = 0;
  size_t best_pool = SIZE_MAX;
  for (int i = 0; i < np; ++i) {
    size_t cnt = 0;
    for (int id : data_nodes)
      if (p.nodes[i].satisfied_by(pcg.g.node(id).label.op)) ++cnt;
    if (cnt < best_pool) {
      best_pool = cnt;
      anchor = i;
    }
  }
  std::vector<int> order{anchor};
  std::vector<bool> in_order(np, false);
  in_order[anchor] = true;
  for (size_t k = 0; k < order.size(); ++k) {
    int i = order[k];
    for (auto const& v : p.inputs[i])
      if (!v.is_input() && !in_order[v.node]) {
        in_order[v.node] = true;
        order.push_back(v.node);
      }
    for (auto const& u : pusers[i])
      if (!in_order[u.first]) {
        in_order[u.first] = true;
        order.push_back(u.first);
      }
  }
  if (static_cast<int>(order.size()) != np) throw FFError("find_pattern_matches: pattern is not connected");

  std::vector<int> assign(np, -1);
  std::vector<ValueRef> imap(p.num_inputs, ValueRef{-1, 0});
  std::set<int> used;

  auto node_ok = [&](int pi, int id) -> bool {
    if (used.count(id) || weight_path[id]) return false;
    auto const& n = pcg.g.node(id);
    if (n.label.op.type == OpType::INPUT) return false;
    if (!p.nodes[pi].satisfied_by(n.label.op)) return false;
    auto din = pcg.layer_data_inputs(id);
    if (din.size() != p.inputs[pi].size()) return false;
    return true;
  };
  // bind pi -> id, returns undo info or false
  std::function<void(size_t)> rec = [&](size_t k) {
    if (out.size() >= max_matches) return;
    if (k == order.size()) {
      // internal (non-exposed) outputs must not escape the match
      std::set<int> matched(assign.begin(), assign.end());
      for (int i = 0; i < np; ++i) {
        auto const& n = pcg.g.node(assign[i]);
        for (size_t o = 0; o < n.outputs.size(); ++o) {
          bool exposed = std::find(p.outputs.begin(), p.outputs.end(), PatternValue{i, static_cast<int>(o)}) !=
                         p.outputs.end();
          if (exposed) continue;
          auto it = vusers.find(ValueRef{assign[i], static_cast<int>(o)});
          if (it == vusers.end()) continue;
          for (auto const& u : it->second)
            if (!matched.count(u.first)) return;
        }
      }
      for (auto const& v : imap)
        if (v.node >= 0 && matched.count(v.node)) return;
      out.push_back({assign, imap});
      return;
    }
    int pi = order[k];
    // candidates from an already-assigned neighbour
    std::vector<int> cands;
    bool constrained = false;
    for (size_t s = 0; s < p.inputs[pi].size() && !constrained; ++s) {
      auto const& v = p.inputs[pi][s];
      if (!v.is_input() && assign[v.node] >= 0) {
        constrained = true;
        auto it = vusers.find(ValueRef{assign[v.node], v.idx});
        if (it != vusers.end())
          for (auto const& u : it->second)
            if (u.second == static_cast<int>(s)) cands.push_back(u.first);
      }
    }
    if (!constrained)
      for (auto const& u : pusers[pi]) {
        if (assign[u.first] < 0) continue;
        constrained = true;
        auto const& in = pcg.g.node(assign[u.first]).inputs;
        if (u.second < static_cast<int>(in.size())) cands.push_back(in[u.second].node);
        break;
      }
    if (!constrained) cands = data_nodes;
    for (int id : cands) {
      if (!node_ok(pi, id)) continue;
      auto din = pcg.layer_data_inputs(id);
      // check every edge touching pi against assigned neighbours / inputs
      std::vector<int> newly_bound;
      bool ok = true;
      for (size_t s = 0; s < din.size() && ok; ++s) {
        auto const& v = p.inputs[pi][s];
        if (v.is_input()) {
          auto& slot = imap[v.input_index()];
          if (slot.node < 0) {
            slot = din[s];
            newly_bound.push_back(v.input_index());
          } else if (!(slot == din[s])) {
            ok = false;
          }
        } else if (assign[v.node] >= 0) {
          if (!(din[s] == ValueRef{assign[v.node], v.idx})) ok = false;
        }
      }
      for (auto const& u : pusers[pi]) {
        if (!ok) break;
        if (assign[u.first] < 0) continue;
        auto const& in = pcg.g.node(assign[u.first]).inputs;
        auto const& pv = p.inputs[u.first][u.second];
        if (u.second >= static_cast<int>(in.size()) || !(in[u.second] == ValueRef{id, pv.idx})) ok = false;
      }
      if (ok) {
        assign[pi] = id;
        used.insert(id);
        rec(k + 1);
        used.erase(id);
        assign[pi] = -1;
      }
      for (int b : newly_bound) imap[b] = ValueRef{-1, 0};
    }
  };
  rec(0);
  return out;
}

// ---------------------------------------------------------------------------
// application
static int weight_root(const ParallelComputationGraph& pcg, ValueRef v) {
  int n = v.node;
  while (pcg.g.node(n).label.op.type != OpType::WEIGHT) n = pcg.g.node(n).inputs.at(0).node;
  return n;
}

void remove_dead_parallel_nodes(ParallelComputationGraph& pcg) {
  bool changed = true;
  while (changed) {
    changed = false;
    std::set<int> used;
    for (int id : pcg.g.node_ids())
      for (auto const& v : pcg.g.node(id).inputs) used.insert(v.node);
    for (int id : pcg.g.node_ids()) {
      if (used.count(id)) continue;
      auto t = pcg.g.node(id).label.op.type;
      if (t == OpType::WEIGHT || (is_parallel_op(t) && pcg.is_weight_path(id))) {
        pcg.g.remove_node(id);
        changed = true;
      }
    }
  }
}

std::optional<ParallelComputationGraph> apply_substitution(const ParallelComputationGraph& pcg,
                                                           const Substitution& s, const PCGPatternMatch& m) {
  ParallelComputationGraph out = pcg;
  std::vector<std::vector<ValueRef>> made(s.out_nodes.size());
  auto resolve = [&](const PatternValue& v) -> ValueRef {
    if (v.is_input()) return m.input_map.at(v.input_index());
    return made.at(v.node).at(v.idx);
  };
  try {
    for (size_t k = 0; k < s.out_nodes.size(); ++k) {
      auto const& o = s.out_nodes[k];
      OpAttrs op;
      std::string name = o.name;
      int orig = -1;
      if (o.copy_from >= 0) {
        orig = m.node_map.at(o.copy_from);
        op = pcg.g.node(orig).label.op;
        if (name.empty()) name = pcg.g.node(orig).label.name;
      } else {
        op = OpAttrs(o.type);
      }
      for (auto const& a : o.assign) {
        if (a.copy) op.attrs[a.key] = pcg.g.node(m.node_map.at(a.from_node)).label.op.attrs.at(a.from_key);
        else op.attrs[a.key] = a.value;
      }
      std::vector<ValueRef> ins;
      for (auto const& v : o.inputs) ins.push_back(resolve(v));
      if ((op.type == OpType::REPARTITION || op.type == OpType::COMBINE) && op.i("dim") < 0)
        op.set("dim", op.i("dim") + out.shape(ins.at(0)).num_dims());
      op = normalize_attrs(op);
      int nw = num_weights(op);
      if (nw > 0) {
        std::vector<ParallelTensorShape> ps;
        for (auto const& v : ins) ps.push_back(out.shape(v));
        auto wshapes = infer_parallel_weight_shapes(op, ps);
        std::vector<ValueRef> ow;
        if (orig >= 0) ow = pcg.layer_weights(orig);
        auto wn = weight_names(op);
        for (int i = 0; i < nw; ++i) {
          if (i < static_cast<int>(ow.size())) {
            int root = weight_root(pcg, ow[i]);
            auto const& rn = pcg.g.node(root);
            ins.push_back(out.add_weight(rn.outputs[0].shape.reduced_shape(), wshapes[i],
                                         rn.outputs[0].initializer, rn.outputs[0].create_grad, rn.label.name));
          } else {
            ins.push_back(out.add_weight(wshapes[i].reduced_shape(), wshapes[i],
                                         default_initializer(op.type, wn.at(i)), true, name + "." + wn.at(i)));
          }
        }
      }
      made[k] = out.add_layer(op, ins, name);
    }
  } catch (const FFError&) {
    return std::nullopt;
  }
  for (size_t j = 0; j < s.pattern.outputs.size(); ++j) {
    auto const& pv = s.pattern.outputs[j];
    ValueRef old{m.node_map.at(pv.node), pv.idx};
    ValueRef nw = resolve(s.output_mapping.at(j));
    if (out.shape(nw) != pcg.shape(old)) return std::nullopt;
    out.g.replace_uses(old, nw);
  }
  for (int id : m.node_map) out.g.remove_node(id);
  remove_dead_parallel_nodes(out);
  return out;
}

// ---------------------------------------------------------------------------
// built-in rules
namespace {

OutputOperator new_op(OpType t, std::vector<PatternValue> ins, std::vector<std::pair<std::string, AttrValue>> kv) {
  OutputOperator o;
  o.type = t;
  o.inputs = std::move(ins);
  for (auto& x : kv) o.assign.push_back({x.first, false, -1, "", x.second});
  return o;
}

OutputOperator copy_op(int from, std::vector<PatternValue> ins) {
  OutputOperator o;
  o.copy_from = from;
  o.inputs = std::move(ins);
  return o;
}

// T(x_0..x_{n-1}) -> [pre_i(x_i)] -> T -> [post_j] with per-input/output wrappers
Substitution wrap_rule(const std::string& name, OpType t, int n_in, int n_out,
                       const std::function<std::vector<OutputOperator>(PatternValue, int)>& pre,
                       const std::function<std::vector<OutputOperator>(PatternValue, int)>& post,
                       std::vector<AttrConstraint> cons = {}) {
  Substitution s;
  s.name = name;
  OperatorPattern op;
  op.type = t;
  op.attrs = std::move(cons);
  std::vector<PatternValue> ins;
  for (int i = 0; i < n_in; ++i) ins.push_back(PatternValue::input(i));
  s.pattern.add_node(op, ins);
  for (int j = 0; j < n_out; ++j) s.pattern.outputs.push_back({0, j});
  std::vector<PatternValue> new_ins;
  for (int i = 0; i < n_in; ++i) {
    PatternValue cur = PatternValue::input(i);
    for (auto o : pre(cur, i)) {
      o.inputs = {cur};
      s.out_nodes.push_back(o);
      cur = {static_cast<int>(s.out_nodes.size()) - 1, 0};
    }
    new_ins.push_back(cur);
  }
  s.out_nodes.push_back(copy_op(0, new_ins));
  int core = static_cast<int>(s.out_nodes.size()) - 1;
  for (int j = 0; j < n_out; ++j) {
    PatternValue cur{core, j};
    for (auto o : post(cur, j)) {
      o.inputs = {cur};
      s.out_nodes.push_back(o);
      cur = {static_cast<int>(s.out_nodes.size()) - 1, 0};
    }
    s.output_mapping.push_back(cur);
  }
  return s;
}

Substitution cancel_rule(const std::string& name, OpType first, OpType second, int degree, bool same_dim) {
  // second(first(x)) -> x   (dims equal when same_dim)
  Substitution s;
  s.name = name;
  OperatorPattern a, b;
  a.type = first;
  b.type = second;
  a.attrs.push_back({AttrConstraint::EQUAL, "degree", int64_t(degree)});
  b.attrs.push_back({AttrConstraint::EQUAL, "degree", int64_t(degree)});
  (void)same_dim;
  s.pattern.add_node(a, {PatternValue::input(0)});
  s.pattern.add_node(b, {{0, 0}});
  s.pattern.outputs.push_back({1, 0});
  s.output_mapping.push_back(PatternValue::input(0));
  return s;
}

}  // namespace

std::vector<Substitution> generate_parallelization_substitutions(const ParallelComputationGraph& pcg, int world) {
  std::vector<Substitution> rules;
  // distinct (op type, #data inputs, #outputs, rank) among compute ops
  std::set<std::tuple<OpType, int, int>> kinds;
  std::set<int> ranks;
  for (int id : pcg.g.node_ids()) {
    auto const& n = pcg.g.node(id);
    auto t = n.label.op.type;
    if (t == OpType::INPUT || t == OpType::WEIGHT || is_parallel_op(t)) continue;
    kinds.insert({t, static_cast<int>(pcg.layer_data_inputs(id).size()), static_cast<int>(n.outputs.size())});
    for (auto const& o : n.outputs) ranks.insert(o.shape.num_dims());
  }
  for (int d = 2; d <= world; ++d) {
    if (world % d) continue;
    const int64_t D = d;
    for (auto const& k : kinds) {
      OpType t = std::get<0>(k);
      int ni = std::get<1>(k), no = std::get<2>(k);
      rules.push_back(wrap_rule(
          "partition_sample_" + to_string(t) + "_" + std::to_string(d), t, ni, no,
          [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REPARTITION, {}, {{"dim", int64_t(0)}, {"degree", D}})}; },
          [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::COMBINE, {}, {{"dim", int64_t(0)}, {"degree", D}})}; }));
      if (t == OpType::LINEAR || (t == OpType::EMBEDDING)) {
        rules.push_back(wrap_rule(
            "column_parallel_" + to_string(t) + "_" + std::to_string(d), t, 1, 1,
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REPLICATE, {}, {{"degree", D}})}; },
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::COMBINE, {}, {{"dim", int64_t(-1)}, {"degree", D}})}; }));
      }
      if (t == OpType::LINEAR) {
        rules.push_back(wrap_rule(
            "row_parallel_LINEAR_" + std::to_string(d), t, 1, 1,
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REPARTITION, {}, {{"dim", int64_t(-1)}, {"degree", D}})}; },
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REDUCTION, {}, {{"degree", D}})}; },
            {{AttrConstraint::EQUAL, "activation", std::string("none")}}));
      }
      // trade d of the sample-dim degree for model parallelism (keeps the
      // total degree, so they apply on top of a data-parallel PCG)
      auto trade_pre = [&](OpType rep_kind) {
        return [&, rep_kind](PatternValue, int) {
          std::vector<OutputOperator> v{new_op(OpType::COMBINE, {}, {{"dim", int64_t(0)}, {"degree", D}})};
          if (rep_kind == OpType::REPLICATE) v.push_back(new_op(OpType::REPLICATE, {}, {{"degree", D}}));
          else v.push_back(new_op(OpType::REPARTITION, {}, {{"dim", int64_t(-1)}, {"degree", D}}));
          return v;
        };
      };
      if (t == OpType::LINEAR || t == OpType::EMBEDDING) {
        rules.push_back(wrap_rule(
            "trade_sample_for_column_" + to_string(t) + "_" + std::to_string(d), t, 1, 1, trade_pre(OpType::REPLICATE),
            [&](PatternValue, int) {
              return std::vector<OutputOperator>{new_op(OpType::COMBINE, {}, {{"dim", int64_t(-1)}, {"degree", D}}),
                                                 new_op(OpType::REPARTITION, {}, {{"dim", int64_t(0)}, {"degree", D}})};
            }));
      }
      if (t == OpType::LINEAR) {
        rules.push_back(wrap_rule(
            "trade_sample_for_row_LINEAR_" + std::to_string(d), t, 1, 1, trade_pre(OpType::REPARTITION),
            [&](PatternValue, int) {
              return std::vector<OutputOperator>{new_op(OpType::REDUCTION, {}, {{"degree", D}}),
                                                 new_op(OpType::REPARTITION, {}, {{"dim", int64_t(0)}, {"degree", D}})};
            },
            {{AttrConstraint::EQUAL, "activation", std::string("none")}}));
      }
      if (t == OpType::MULTIHEAD_ATTENTION) {
        rules.push_back(wrap_rule(
            "trade_sample_for_heads_MHA_" + std::to_string(d), t, 3, 1, trade_pre(OpType::REPLICATE),
            [&](PatternValue, int) {
              return std::vector<OutputOperator>{new_op(OpType::REDUCTION, {}, {{"degree", D}}),
                                                 new_op(OpType::REPARTITION, {}, {{"dim", int64_t(0)}, {"degree", D}})};
            },
            {{AttrConstraint::DIVISIBLE_BY, "num_heads", D}}));
      }
      if (t == OpType::MULTIHEAD_ATTENTION) {
        rules.push_back(wrap_rule(
            "head_parallel_MHA_" + std::to_string(d), t, 3, 1,
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REPLICATE, {}, {{"degree", D}})}; },
            [&](PatternValue, int) { return std::vector<OutputOperator>{new_op(OpType::REDUCTION, {}, {{"degree", D}})}; },
            {{AttrConstraint::DIVISIBLE_BY, "num_heads", D}}));
      }
    }
    // cancellations (any rank; dims checked through shape equality on apply)
    for (int r : ranks)
      for (int dim = 0; dim < r; ++dim) {
        auto c1 = cancel_rule("cancel_combine_repartition_d" + std::to_string(dim) + "_" + std::to_string(d),
                              OpType::COMBINE, OpType::REPARTITION, d, true);
        c1.pattern.nodes[0].attrs.push_back({AttrConstraint::EQUAL, "dim", int64_t(dim)});
        c1.pattern.nodes[1].attrs.push_back({AttrConstraint::EQUAL, "dim", int64_t(dim)});
        rules.push_back(c1);
        auto c2 = cancel_rule("cancel_repartition_combine_d" + std::to_string(dim) + "_" + std::to_string(d),
                              OpType::REPARTITION, OpType::COMBINE, d, true);
        c2.pattern.nodes[0].attrs.push_back({AttrConstraint::EQUAL, "dim", int64_t(dim)});
        c2.pattern.nodes[1].attrs.push_back({AttrConstraint::EQUAL, "dim", int64_t(dim)});
        rules.push_back(c2);
      }
  }
  // deduplicate cancellation rules produced for several ranks
  std::set<std::string> seen;
  std::vector<Substitution> uniq;
  for (auto& r : rules)
    if (seen.insert(r.name).second) uniq.push_back(std::move(r));
  return uniq;
}

// ---------------------------------------------------------------------------
// legacy corpus
int LegacyOperator::param(const std::string& k, int dflt) const {
  for (auto const& p : params)
    if (p.first == k) return p.second;
  return dflt;
}

LegacyRuleCollection load_legacy_rules(const Json& j) {
  LegacyRuleCollection c;
  auto parse_ops = [](const Json& arr) {
    std::vector<LegacyOperator> ops;
    for (auto const& o : arr.as_array()) {
      LegacyOperator op;
      op.type = o.at("type").as_string();
      for (auto const& t : o.at("input").as_array())
        op.inputs.push_back({static_cast<int>(t.at("opId").as_int()), static_cast<int>(t.at("tsId").as_int())});
      for (auto const& p : o.at("para").as_array())
        op.params.push_back({p.at("key").as_string(), static_cast<int>(p.at("value").as_int())});
      ops.push_back(op);
    }
    return ops;
  };
  for (auto const& r : j.at("rule").as_array()) {
    LegacyRule rule;
    rule.name = r.contains("name") ? r.at("name").as_string() : "";
    rule.src = parse_ops(r.at("srcOp"));
    rule.dst = parse_ops(r.at("dstOp"));
    for (auto const& m : r.at("mappedOutput").as_array())
      rule.mapped_outputs.push_back({static_cast<int>(m.at("srcOpId").as_int()),
                                     static_cast<int>(m.at("srcTsId").as_int()),
                                     static_cast<int>(m.at("dstOpId").as_int()),
                                     static_cast<int>(m.at("dstTsId").as_int())});
    c.rules.push_back(rule);
  }
  return c;
}

std::string legacy_rule_to_dot(const LegacyRule& r) {
  std::ostringstream os;
  os << "digraph \"" << r.name << "\" {\n  compound=true;\n";
  auto side = [&](const char* tag, const std::vector<LegacyOperator>& ops) {
    os << "  subgraph cluster_" << tag << " {\n    label=\"" << tag << "\";\n";
    std::set<int> ext;
    for (size_t i = 0; i < ops.size(); ++i) {
      os << "    " << tag << i << " [shape=box, label=\"" << ops[i].type;
      for (auto const& p : ops[i].params) os << "\\n" << p.first << "=" << p.second;
      os << "\"];\n";
      for (auto const& t : ops[i].inputs)
        if (t.op_id < 0) ext.insert(t.op_id);
    }
    for (int e : ext) os << "    " << tag << "_in" << -e << " [shape=ellipse, label=\"input " << -e << "\"];\n";
    for (size_t i = 0; i < ops.size(); ++i)
      for (auto const& t : ops[i].inputs) {
        if (t.op_id < 0) os << "    " << tag << "_in" << -t.op_id << " -> " << tag << i << ";\n";
        else os << "    " << tag << t.op_id << " -> " << tag << i << " [label=\"" << t.ts_id << "\"];\n";
      }
    os << "  }\n";
  };
  side("src", r.src);
  side("dst", r.dst);
  for (auto const& m : r.mapped_outputs)
    os << "  src" << m.src_op << " -> dst" << m.dst_op << " [style=dashed, constraint=false];\n";
  os << "}\n";
  return os.str();
}

std::optional<Substitution> substitution_from_legacy_rule(const LegacyRule& r) {
  // TASO ActiMode: 0 none, 1 sigmoid, 2 relu, 3 tanh
  auto acti = [](int v) -> std::string {
    switch (v) {
      case 0: return "none";
      case 1: return "sigmoid";
      case 2: return "relu";
      case 3: return "tanh";
      default: return "";
    }
  };
  struct Conv {
    OpType t;
    std::vector<std::pair<std::string, AttrValue>> kv;
    bool ok = true;
  };
  auto conv = [&](const LegacyOperator& o) {
    Conv c{OpType::NOOP, {}};
    const std::string& ty = o.type;
    int dim = o.param("PM_PARALLEL_DIM"), deg = o.param("PM_PARALLEL_DEGREE");
    if (ty == "OP_PARTITION") c = {OpType::REPARTITION, {{"dim", int64_t(-(dim + 1))}, {"degree", int64_t(deg)}}};
    else if (ty == "OP_COMBINE") c = {OpType::COMBINE, {{"dim", int64_t(-(dim + 1))}, {"degree", int64_t(deg)}}};
    else if (ty == "OP_REPLICATE") c = {OpType::REPLICATE, {{"degree", int64_t(deg)}}};
    else if (ty == "OP_REDUCE") c = {OpType::REDUCTION, {{"degree", int64_t(deg)}}};
    else if (ty == "OP_RELU") c = {OpType::RELU, {}};
    else if (ty == "OP_EW_ADD") c = {OpType::EW_ADD, {}};
    else if (ty == "OP_EW_MUL") c = {OpType::EW_MUL, {}};
    else if (ty == "OP_LINEAR") {
      std::string a = acti(o.param("PM_ACTI", 0));
      c = {OpType::LINEAR, {{"activation", a}}};
      c.ok = !a.empty();
    } else if (ty == "OP_CONCAT") c = {OpType::CONCAT, {}};
    else if (ty == "OP_SPLIT") c = {OpType::SPLIT, {}};
    else c.ok = false;
    return c;
  };
  // pattern inputs that feed a LINEAR's weight slot are implicit weights
  std::set<int> weight_ids;
  for (auto const* side : {&r.src, &r.dst})
    for (auto const& o : *side)
      if (o.type == "OP_LINEAR" && o.inputs.size() >= 2) {
        if (o.inputs[1].op_id >= 0) return std::nullopt;  // weight produced by an op: not expressible
        weight_ids.insert(o.inputs[1].op_id);
      }
  for (auto const* side : {&r.src, &r.dst})
    for (auto const& o : *side)
      for (size_t s = 0; s < o.inputs.size(); ++s)
        if (weight_ids.count(o.inputs[s].op_id) && !(o.type == "OP_LINEAR" && s == 1)) return std::nullopt;
  std::map<int, int> in_index;  // legacy negative id -> pattern input index
  auto pin = [&](int legacy_id) {
    auto it = in_index.find(legacy_id);
    if (it != in_index.end()) return it->second;
    int k = static_cast<int>(in_index.size());
    in_index[legacy_id] = k;
    return k;
  };
  Substitution s;
  s.name = "legacy_" + r.name;
  std::map<OpType, int> first_src_of_type;
  for (size_t i = 0; i < r.src.size(); ++i) {
    auto c = conv(r.src[i]);
    if (!c.ok) return std::nullopt;
    OperatorPattern op;
    op.type = c.t;
    for (auto const& kv : c.kv)
      if (kv.first != "dim") op.attrs.push_back({AttrConstraint::EQUAL, kv.first, kv.second});
    std::vector<PatternValue> ins;
    for (size_t k = 0; k < r.src[i].inputs.size(); ++k) {
      if (c.t == OpType::LINEAR && k == 1) continue;
      auto const& t = r.src[i].inputs[k];
      ins.push_back(t.op_id < 0 ? PatternValue::input(pin(t.op_id)) : PatternValue{t.op_id, t.ts_id});
    }
    s.pattern.add_node(op, ins);
    first_src_of_type.emplace(c.t, static_cast<int>(i));
  }
  for (size_t i = 0; i < r.dst.size(); ++i) {
    auto c = conv(r.dst[i]);
    if (!c.ok) return std::nullopt;
    OutputOperator o;
    bool needs_copy = c.t == OpType::LINEAR || c.t == OpType::CONCAT || c.t == OpType::SPLIT;
    if (needs_copy) {
      auto it = first_src_of_type.find(c.t);
      if (it == first_src_of_type.end()) return std::nullopt;
      o.copy_from = it->second;
    } else {
      o.type = c.t;
    }
    for (auto const& kv : c.kv) o.assign.push_back({kv.first, false, -1, "", kv.second});
    for (size_t k = 0; k < r.dst[i].inputs.size(); ++k) {
      if (c.t == OpType::LINEAR && k == 1) continue;
      auto const& t = r.dst[i].inputs[k];
      if (t.op_id < 0) {
        if (!in_index.count(t.op_id)) return std::nullopt;
        o.inputs.push_back(PatternValue::input(in_index.at(t.op_id)));
      } else {
        o.inputs.push_back({t.op_id, t.ts_id});
      }
    }
    s.out_nodes.push_back(o);
  }
  for (auto const& m : r.mapped_outputs) {
    s.pattern.outputs.push_back({m.src_op, m.src_ts});
    s.output_mapping.push_back({m.dst_op, m.dst_ts});
  }
  // the pattern must be connected for matching
  if (s.pattern.nodes.empty()) return std::nullopt;
  std::vector<int> comp(s.pattern.nodes.size());
  for (size_t i = 0; i < comp.size(); ++i) comp[i] = static_cast<int>(i);
  std::function<int(int)> f = [&](int x) { return comp[x] == x ? x : comp[x] = f(comp[x]); };
  for (size_t i = 0; i < s.pattern.nodes.size(); ++i)
    for (auto const& v : s.pattern.inputs[i])
      if (!v.is_input()) comp[f(static_cast<int>(i))] = f(v.node);
  for (size_t i = 0; i < comp.size(); ++i)
    if (f(static_cast<int>(i)) != f(0)) return std::nullopt;
  return s;
}

}  // namespace ff
