#include "ff/substitution.h"

#include <algorithm>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>

namespace ff {

// ---------------------------------------------------------------------------
// patterns
bool OperatorPattern::satisfied_by(const OpAttrs& op, int rank) const {
  if (type && op.type != *type) return false;
  for (auto const& c : attrs) {
    auto it = op.attrs.find(c.key);
    if (it == op.attrs.end()) return false;
    if (c.kind == AttrConstraint::EQUAL) {
      if (it->second != c.value) return false;
    } else if (c.kind == AttrConstraint::DIM_FROM_END) {
      if (rank <= 0 || !std::holds_alternative<int64_t>(it->second) || !std::holds_alternative<int64_t>(c.value))
        return false;
      int64_t have = std::get<int64_t>(it->second), want = std::get<int64_t>(c.value) + rank;
      if (have < 0) have += rank;
      if (want < 0 || have != want) return false;
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
static PatternValue pv_from(const Json& j) {
  auto const& a = j.as_array();
  return {static_cast<int>(a.at(0).as_int()), static_cast<int>(a.at(1).as_int())};
}
static const char* kind_name(AttrConstraint::Kind k) {
  switch (k) {
    case AttrConstraint::EQUAL: return "equal";
    case AttrConstraint::DIVISIBLE_BY: return "divisible_by";
    case AttrConstraint::DIM_FROM_END: return "dim_from_end";
  }
  return "equal";
}
static AttrConstraint::Kind kind_from(const std::string& s) {
  if (s == "equal") return AttrConstraint::EQUAL;
  if (s == "divisible_by") return AttrConstraint::DIVISIBLE_BY;
  if (s == "dim_from_end") return AttrConstraint::DIM_FROM_END;
  throw FFError("substitution json: unknown constraint kind '" + s + "'");
}

// Format "ffmi355x.substitution.v1": lossless (every constraint kind, output
// operator provenance, names), so rule sets can be stored, exchanged and
// reloaded (load_substitutions).  "attrs" / "assign" keep the readable
// one-line summaries the dot exporter and reports use.
Json Substitution::to_json() const {
  Json j = Json::object();
  j["format"] = "ffmi355x.substitution.v1";
  j["name"] = name;
  Json pn = Json::array();
  for (size_t i = 0; i < pattern.nodes.size(); ++i) {
    auto const& nd = pattern.nodes[i];
    Json n = Json::object();
    n["type"] = nd.type ? to_string(*nd.type) : "*";
    Json c = Json::object();
    Json cons = Json::array();
    for (auto const& a : nd.attrs) {
      c[a.key] = attr_to_json(a.value);
      Json x = Json::object();
      x["kind"] = kind_name(a.kind);
      x["key"] = a.key;
      x["value"] = attr_to_json(a.value);
      cons.push_back(x);
    }
    n["attrs"] = c;
    n["constraints"] = cons;
    n["num_outputs"] = static_cast<int64_t>(nd.num_outputs);
    Json ins = Json::array();
    for (auto const& v : pattern.inputs[i]) ins.push_back(pv_json(v));
    n["inputs"] = ins;
    pn.push_back(n);
  }
  j["pattern"] = pn;
  j["num_pattern_inputs"] = static_cast<int64_t>(pattern.num_inputs);
  Json po = Json::array();
  for (auto const& v : pattern.outputs) po.push_back(pv_json(v));
  j["pattern_outputs"] = po;
  Json on = Json::array();
  for (auto const& o : out_nodes) {
    Json n = Json::object();
    n["type"] = o.copy_from >= 0 ? "copy_of_" + std::to_string(o.copy_from) : to_string(o.type);
    n["copy_from"] = static_cast<int64_t>(o.copy_from);
    n["op_type"] = to_string(o.type);
    n["name"] = o.name;
    Json a = Json::object();
    Json al = Json::array();
    for (auto const& x : o.assign) {
      a[x.key] = x.copy ? Json("copy:" + std::to_string(x.from_node) + "." + x.from_key) : attr_to_json(x.value);
      Json y = Json::object();
      y["key"] = x.key;
      y["copy"] = x.copy;
      y["from_node"] = static_cast<int64_t>(x.from_node);
      y["from_key"] = x.from_key;
      if (!x.copy) y["value"] = attr_to_json(x.value);
      al.push_back(y);
    }
    n["assign"] = a;
    n["assignments"] = al;
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

Substitution Substitution::from_json(const Json& j) {
  Substitution s;
  s.name = j.at("name").as_string();
  for (auto const& n : j.at("pattern").as_array()) {
    OperatorPattern op;
    std::string t = n.at("type").as_string();
    if (t != "*") op.type = optype_from_string(t);
    for (auto const& c : n.at("constraints").as_array())
      op.attrs.push_back({kind_from(c.at("kind").as_string()), c.at("key").as_string(), attr_from_json(c.at("value"))});
    std::vector<PatternValue> ins;
    for (auto const& v : n.at("inputs").as_array()) ins.push_back(pv_from(v));
    int no = n.contains("num_outputs") ? static_cast<int>(n.at("num_outputs").as_int()) : -1;
    s.pattern.add_node(op, ins);
    s.pattern.nodes.back().num_outputs = no;
  }
  if (j.contains("num_pattern_inputs"))
    s.pattern.num_inputs = std::max(s.pattern.num_inputs, static_cast<int>(j.at("num_pattern_inputs").as_int()));
  for (auto const& v : j.at("pattern_outputs").as_array()) s.pattern.outputs.push_back(pv_from(v));
  for (auto const& n : j.at("output_graph").as_array()) {
    OutputOperator o;
    o.copy_from = static_cast<int>(n.at("copy_from").as_int());
    o.type = optype_from_string(n.at("op_type").as_string());
    o.name = n.contains("name") ? n.at("name").as_string() : "";
    for (auto const& y : n.at("assignments").as_array()) {
      AttrAssignment a;
      a.key = y.at("key").as_string();
      a.copy = y.at("copy").as_bool();
      a.from_node = static_cast<int>(y.at("from_node").as_int());
      a.from_key = y.at("from_key").as_string();
      if (!a.copy) a.value = attr_from_json(y.at("value"));
      o.assign.push_back(a);
    }
    for (auto const& v : n.at("inputs").as_array()) o.inputs.push_back(pv_from(v));
    s.out_nodes.push_back(o);
  }
  for (auto const& v : j.at("output_mapping").as_array()) s.output_mapping.push_back(pv_from(v));
  return s;
}

// ---------------------------------------------------------------------------
// matching
// Backtracking search over pattern nodes in an order where every node after
// the first of its weakly-connected component is adjacent to an earlier one
// (its candidates come from the already-bound neighbour); a component's first
// node takes its candidates from a pattern input another component already
// bound, else from its own pool.  Disconnected patterns (the legacy corpus
// has rules over independent operators that only share, or do not even
// share, inputs -- the reference splits and merges such patterns,
// find_pattern_matches.cc:70-115) are the product of their components' matches.
PatternMatchIndex::PatternMatchIndex(const ParallelComputationGraph& pcg) {
  const int n_ids = pcg.g.next_id();
  weight_path.assign(n_ids, 0);
  rank.assign(n_ids, -1);
  din.resize(n_ids);
  users.resize(n_ids);
  for (int id : pcg.g.topo_order()) {
    auto const& n = pcg.g.node(id);
    users[id].resize(n.outputs.size());
    weight_path[id] = pcg.is_weight_path(id);
    if (!weight_path[id] && n.label.op.type != OpType::INPUT) {
      data_nodes.push_back(id);
      by_type[n.label.op.type].push_back(id);
      din[id] = pcg.layer_data_inputs(id);
      rank[id] = din[id].empty() ? -1 : pcg.shape(din[id][0]).num_dims();
    }
  }
  for (int id : pcg.g.node_ids()) {
    auto const& n = pcg.g.node(id);
    for (size_t s = 0; s < n.inputs.size(); ++s) {
      auto const& v = n.inputs[s];
      if (v.node >= 0 && v.node < n_ids && v.idx < static_cast<int>(users[v.node].size()))
        users[v.node][v.idx].push_back({id, static_cast<int>(s)});
    }
  }
}

const std::vector<std::pair<int, int>>& PatternMatchIndex::users_of(const ValueRef& v) const {
  static const std::vector<std::pair<int, int>> none;
  if (v.node < 0 || v.node >= static_cast<int>(users.size()) || v.idx >= static_cast<int>(users[v.node].size()))
    return none;
  return users[v.node][v.idx];
}

std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  size_t max_matches) {
  return find_pattern_matches(p, pcg, PatternMatchIndex(pcg), max_matches);
}

std::vector<PCGPatternMatch> find_pattern_matches(const PCGPattern& p, const ParallelComputationGraph& pcg,
                                                  const PatternMatchIndex& ix, size_t max_matches) {
  std::vector<PCGPatternMatch> out;
  const int np = static_cast<int>(p.nodes.size());
  if (np == 0) return out;
  auto fits = [&](int pi, int id) -> bool {
    auto const& n = pcg.g.node(id);
    if (!p.nodes[pi].satisfied_by(n.label.op, ix.rank[id])) return false;
    if (p.nodes[pi].num_outputs >= 0 && static_cast<int>(n.outputs.size()) != p.nodes[pi].num_outputs) return false;
    return ix.din[id].size() == p.inputs[pi].size();
  };
  std::vector<std::vector<int>> pool(np);
  for (int i = 0; i < np; ++i) {
    const std::vector<int>* cand = &ix.data_nodes;
    if (p.nodes[i].type) {
      auto it = ix.by_type.find(*p.nodes[i].type);
      if (it == ix.by_type.end()) return out;
      cand = &it->second;
    }
    for (int id : *cand)
      if (fits(i, id)) pool[i].push_back(id);
    if (pool[i].empty()) return out;
  }
  std::vector<std::vector<std::pair<int, int>>> pusers(np);  // pattern node -> (user pnode, slot)
  for (int i = 0; i < np; ++i)
    for (size_t s = 0; s < p.inputs[i].size(); ++s)
      if (!p.inputs[i][s].is_input()) pusers[p.inputs[i][s].node].push_back({i, static_cast<int>(s)});
  // order: BFS per component; next component preferably one sharing a bound input
  std::vector<int> order;
  std::vector<bool> in_order(np, false);
  std::set<int> bound_inputs;
  while (static_cast<int>(order.size()) < np) {
    int anchor = -1;
    size_t best = SIZE_MAX;
    bool best_shares = false;
    for (int i = 0; i < np; ++i) {
      if (in_order[i]) continue;
      bool shares = false;
      for (auto const& v : p.inputs[i])
        if (v.is_input() && bound_inputs.count(v.input_index())) shares = true;
      if ((shares && !best_shares) || (shares == best_shares && pool[i].size() < best)) {
        anchor = i;
        best = pool[i].size();
        best_shares = shares;
      }
    }
    size_t k = order.size();
    order.push_back(anchor);
    in_order[anchor] = true;
    for (; k < order.size(); ++k) {
      int i = order[k];
      for (auto const& v : p.inputs[i]) {
        if (v.is_input()) bound_inputs.insert(v.input_index());
        else if (!in_order[v.node]) {
          in_order[v.node] = true;
          order.push_back(v.node);
        }
      }
      for (auto const& u : pusers[i])
        if (!in_order[u.first]) {
          in_order[u.first] = true;
          order.push_back(u.first);
        }
    }
  }

  std::vector<int> assign(np, -1);
  std::vector<ValueRef> imap(p.num_inputs, ValueRef{-1, 0});
  std::set<int> used;

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
          for (auto const& u : ix.users_of(ValueRef{assign[i], static_cast<int>(o)}))
            if (!matched.count(u.first)) return;
        }
      }
      for (auto const& v : imap)
        if (v.node >= 0 && matched.count(v.node)) return;
      out.push_back({assign, imap});
      return;
    }
    int pi = order[k];
    // candidates from an already-bound neighbour or pattern input
    std::vector<int> cands;
    bool constrained = false;
    for (size_t s = 0; s < p.inputs[pi].size() && !constrained; ++s) {
      auto const& v = p.inputs[pi][s];
      ValueRef src{-1, 0};
      if (!v.is_input() && assign[v.node] >= 0) src = ValueRef{assign[v.node], v.idx};
      else if (v.is_input() && imap[v.input_index()].node >= 0) src = imap[v.input_index()];
      if (src.node < 0) continue;
      constrained = true;
      for (auto const& u : ix.users_of(src))
        if (u.second == static_cast<int>(s)) cands.push_back(u.first);
    }
    if (!constrained)
      for (auto const& u : pusers[pi]) {
        if (assign[u.first] < 0) continue;
        constrained = true;
        auto const& in = pcg.g.node(assign[u.first]).inputs;
        if (u.second < static_cast<int>(in.size())) cands.push_back(in[u.second].node);
        break;
      }
    if (!constrained) cands = pool[pi];
    for (int id : cands) {
      if (used.count(id) || ix.weight_path[id] || pcg.g.node(id).label.op.type == OpType::INPUT) continue;
      if (!fits(pi, id)) continue;
      auto const& din = ix.din[id];
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
      if (out.size() >= max_matches) return;
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
  // use counts + a worklist: removing a dead weight-path node may make its
  // producer dead in turn (reads go through a const view: mutable node
  // access would unshare copy-on-write nodes)
  const ParallelComputationGraph& cg = pcg;
  const int n = cg.g.next_id();
  std::vector<int> uses(n, 0);
  for (int id : cg.g.node_ids())
    for (auto const& v : cg.g.node(id).inputs)
      if (v.node >= 0 && v.node < n) ++uses[v.node];
  auto removable = [&](int id) {
    auto t = cg.g.node(id).label.op.type;
    return t == OpType::WEIGHT || (is_parallel_op(t) && cg.is_weight_path(id));
  };
  std::vector<int> work;
  for (int id : cg.g.node_ids())
    if (uses[id] == 0 && removable(id)) work.push_back(id);
  while (!work.empty()) {
    int id = work.back();
    work.pop_back();
    if (!cg.g.has_node(id)) continue;
    std::vector<ValueRef> ins = cg.g.node(id).inputs;
    pcg.g.remove_node(id);
    for (auto const& v : ins)
      if (v.node >= 0 && v.node < n && --uses[v.node] == 0 && cg.g.has_node(v.node) && removable(v.node))
        work.push_back(v.node);
  }
}

std::optional<ParallelComputationGraph> apply_substitution(const ParallelComputationGraph& pcg,
                                                           const Substitution& s, const PCGPatternMatch& m) {
  // 1. the rewritten operators and their parallel shapes, computed on the
  //    side: most candidate rewrites of a search fail shape inference or the
  //    output-shape check, and those must not pay for a copy of the graph
  std::vector<OpAttrs> ops(s.out_nodes.size());
  std::vector<std::string> names(s.out_nodes.size());
  std::vector<std::vector<ParallelTensorShape>> oshape(s.out_nodes.size());
  auto shape_of = [&](const PatternValue& v) -> const ParallelTensorShape& {
    if (v.is_input()) return pcg.shape(m.input_map.at(v.input_index()));
    return oshape.at(v.node).at(v.idx);
  };
  try {
    for (size_t k = 0; k < s.out_nodes.size(); ++k) {
      auto const& o = s.out_nodes[k];
      OpAttrs op;
      std::string name = o.name;
      if (o.copy_from >= 0) {
        int orig = m.node_map.at(o.copy_from);
        op = pcg.g.node(orig).label.op;
        if (name.empty()) name = pcg.g.node(orig).label.name;
      } else {
        op = OpAttrs(o.type);
      }
      for (auto const& a : o.assign) {
        if (a.copy) op.attrs[a.key] = pcg.g.node(m.node_map.at(a.from_node)).label.op.attrs.at(a.from_key);
        else op.attrs[a.key] = a.value;
      }
      std::vector<ParallelTensorShape> ins;
      for (auto const& v : o.inputs) ins.push_back(shape_of(v));
      if (ins.empty()) return std::nullopt;
      if ((op.type == OpType::REPARTITION || op.type == OpType::COMBINE) && op.i("dim") < 0)
        op.set("dim", op.i("dim") + ins[0].num_dims());
      auto eq = op.attrs.find("_equal_splits");
      if (eq != op.attrs.end()) {
        // a legacy SPLIT states only its number of outputs: equal pieces
        const int64_t n = std::get<int64_t>(eq->second);
        op.attrs.erase(eq);
        int64_t ax = op.i("axis");
        if (ax < 0) ax += ins[0].num_dims();
        if (n <= 0 || ax < 0 || ax >= ins[0].num_dims() || ins[0].shard_dims[ax].size % n) return std::nullopt;
        op.set("splits", std::vector<int64_t>(n, ins[0].shard_dims[ax].size / n));
      }
      op = normalize_attrs(op);
      oshape[k] = infer_parallel_output_shapes(op, ins);
      ops[k] = std::move(op);
      names[k] = name;
    }
    for (size_t j = 0; j < s.pattern.outputs.size(); ++j) {
      auto const& pv = s.pattern.outputs[j];
      if (shape_of(s.output_mapping.at(j)) != pcg.shape(ValueRef{m.node_map.at(pv.node), pv.idx}))
        return std::nullopt;
    }
  } catch (const FFError&) {
    return std::nullopt;
  } catch (const std::out_of_range&) {
    return std::nullopt;
  }

  // 2. the rewrite itself
  ParallelComputationGraph out = pcg;
  std::vector<std::vector<ValueRef>> made(s.out_nodes.size());
  auto resolve = [&](const PatternValue& v) -> ValueRef {
    if (v.is_input()) return m.input_map.at(v.input_index());
    return made.at(v.node).at(v.idx);
  };
  try {
    for (size_t k = 0; k < s.out_nodes.size(); ++k) {
      auto const& o = s.out_nodes[k];
      const OpAttrs& op = ops[k];
      const std::string& name = names[k];
      int orig = o.copy_from >= 0 ? m.node_map.at(o.copy_from) : -1;
      std::vector<ValueRef> ins;
      for (auto const& v : o.inputs) ins.push_back(resolve(v));
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
            // a weight with no matched source would be created fresh: a new
            // name and a default initializer, which drops the user's
            // initializer and breaks get/set of weights by name and checkpoint
            // keys.  Such rewrites are rejected (the TASO corpus is on by
            // default, so this path is reachable in ordinary searches).
            (void)wn;
            return std::nullopt;
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
  // a match whose pattern inputs are reachable from its own outputs (possible
  // across the components of a disconnected pattern) would close a cycle
  try {
    (void)out.g.topo_order();
  } catch (const FFError&) {
    return std::nullopt;
  }
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

// Linear(activation none) followed by an activation operator -> one Linear
// with the activation fused into its epilogue (the reference's substitution
// test case, lib/substitutions/test/src/substitutions/substitution.cc; the
// legacy corpus has it only under parallel operators, e.g. taso_rule_278).
static std::vector<Substitution> activation_fusion_rules() {
  std::vector<Substitution> rules;
  const std::pair<OpType, const char*> acts[] = {
      {OpType::RELU, "relu"}, {OpType::SIGMOID, "sigmoid"}, {OpType::TANH, "tanh"}, {OpType::GELU, "gelu"}};
  for (auto const& a : acts) {
    Substitution s;
    s.name = std::string("fuse_linear_") + a.second;
    OperatorPattern lin, act;
    lin.type = OpType::LINEAR;
    lin.attrs.push_back({AttrConstraint::EQUAL, "activation", std::string("none")});
    act.type = a.first;
    s.pattern.add_node(lin, {PatternValue::input(0)});
    s.pattern.add_node(act, {{0, 0}});
    s.pattern.outputs.push_back({1, 0});
    OutputOperator o = copy_op(0, {PatternValue::input(0)});
    o.assign.push_back({"activation", false, -1, "", std::string(a.second)});
    s.out_nodes.push_back(o);
    s.output_mapping.push_back({0, 0});
    rules.push_back(s);
  }
  return rules;
}

std::vector<Substitution> generate_parallelization_substitutions(const ParallelComputationGraph& pcg, int world) {
  std::vector<Substitution> rules = activation_fusion_rules();
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

std::optional<Substitution> substitution_from_legacy_rule(const LegacyRule& r, std::string* why) {
  auto fail = [&](const std::string& m) -> std::optional<Substitution> {
    if (why) *why = m;
    return std::nullopt;
  };
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
  // legacy dims are innermost-first: dim d is the (d+1)-th from the end
  auto from_end = [](int d) { return static_cast<int64_t>(-(d + 1)); };

  struct Side {
    const std::vector<LegacyOperator>* ops;
    std::vector<bool> weight_only;  // output feeds only Linear weight slots (transitively)
    std::vector<int> remap;         // legacy op index -> kept index (-1 dropped)
  };
  std::set<int> weight_inputs, data_inputs;  // legacy negative ids
  auto analyse = [&](const std::vector<LegacyOperator>& ops, bool is_src, Side& sd) -> std::string {
    const int n = static_cast<int>(ops.size());
    sd.ops = &ops;
    sd.weight_only.assign(n, false);
    std::vector<std::vector<std::pair<int, int>>> users(n);
    for (int j = 0; j < n; ++j)
      for (size_t k = 0; k < ops[j].inputs.size(); ++k) {
        int o = ops[j].inputs[k].op_id;
        if (o >= n) return "forward reference";
        if (o >= 0) users[o].push_back({j, static_cast<int>(k)});
      }
    std::set<int> mapped;
    for (auto const& m : r.mapped_outputs) mapped.insert(is_src ? m.src_op : m.dst_op);
    for (int i = n - 1; i >= 0; --i) {
      if (users[i].empty() || mapped.count(i)) continue;
      bool w = true;
      for (auto const& u : users[i])
        if (!((ops[u.first].type == "OP_LINEAR" && u.second == 1) || sd.weight_only[u.first])) w = false;
      sd.weight_only[i] = w;
    }
    for (int j = 0; j < n; ++j)
      for (size_t k = 0; k < ops[j].inputs.size(); ++k) {
        int o = ops[j].inputs[k].op_id;
        bool weight_slot = (ops[j].type == "OP_LINEAR" && k == 1) || sd.weight_only[j];
        if (o < 0) (weight_slot ? weight_inputs : data_inputs).insert(o);
        else if (weight_slot && !sd.weight_only[o])
          return "a Linear weight computed from data";
      }
    sd.remap.assign(n, -1);
    int kept = 0;
    for (int i = 0; i < n; ++i)
      if (!sd.weight_only[i]) sd.remap[i] = kept++;
    return "";
  };
  Side src, dst;
  std::string e = analyse(r.src, true, src);
  if (e.empty()) e = analyse(r.dst, false, dst);
  if (!e.empty()) return fail(e);
  for (int w : weight_inputs)
    if (data_inputs.count(w)) return fail("a pattern input used both as a weight and as data");
  // weight root of a Linear: the legacy input id its weight chain starts from
  auto weight_root = [](const std::vector<LegacyOperator>& ops, int j) {
    int o = ops[j].inputs.at(1).op_id;
    while (o >= 0) o = ops[o].inputs.at(0).op_id;
    return o;
  };

  struct Conv {
    OpType t = OpType::NOOP;
    std::vector<AttrConstraint> cons;                              // pattern side
    std::vector<std::pair<std::string, AttrValue>> assign;         // output side
    int num_outputs = -1;
  };
  auto conv = [&](const LegacyOperator& o, Conv& c) -> std::string {
    const std::string& ty = o.type;
    int dim = o.param("PM_PARALLEL_DIM"), deg = o.param("PM_PARALLEL_DEGREE");
    if (ty == "OP_PARTITION" || ty == "OP_COMBINE") {
      if (dim < 0 || deg < 1) return "parallel op without dim / degree";
      c.t = ty == "OP_PARTITION" ? OpType::REPARTITION : OpType::COMBINE;
      c.cons = {{AttrConstraint::DIM_FROM_END, "dim", from_end(dim)}, {AttrConstraint::EQUAL, "degree", int64_t(deg)}};
      c.assign = {{"dim", from_end(dim)}, {"degree", int64_t(deg)}};
    } else if (ty == "OP_REPLICATE" || ty == "OP_REDUCE") {
      // the legacy replica dim is implicit in the replica degrees here
      if (deg < 1) return "parallel op without degree";
      c.t = ty == "OP_REPLICATE" ? OpType::REPLICATE : OpType::REDUCTION;
      c.cons = {{AttrConstraint::EQUAL, "degree", int64_t(deg)}};
      c.assign = {{"degree", int64_t(deg)}};
    } else if (ty == "OP_RELU") {
      c.t = OpType::RELU;
    } else if (ty == "OP_EW_ADD") {
      c.t = OpType::EW_ADD;
    } else if (ty == "OP_EW_MUL") {
      c.t = OpType::EW_MUL;
    } else if (ty == "OP_LINEAR") {
      std::string a = acti(o.param("PM_ACTI", 0));
      if (a.empty()) return "unknown activation";
      c.t = OpType::LINEAR;
      c.cons = {{AttrConstraint::EQUAL, "activation", a}};
      c.assign = {{"activation", a}};
    } else if (ty == "OP_CONCAT") {
      int ax = o.param("PM_AXIS");
      if (ax < 0) return "concat without axis";
      c.t = OpType::CONCAT;
      c.cons = {{AttrConstraint::DIM_FROM_END, "axis", from_end(ax)}};
      c.assign = {{"axis", from_end(ax)}};
    } else if (ty == "OP_SPLIT") {
      int ax = o.param("PM_AXIS"), n = o.param("PM_NUM_OUTPUTS");
      if (ax < 0 || n < 1) return "split without axis / outputs";
      c.t = OpType::SPLIT;
      c.cons = {{AttrConstraint::DIM_FROM_END, "axis", from_end(ax)}};
      c.assign = {{"axis", from_end(ax)}, {"_equal_splits", int64_t(n)}};
      c.num_outputs = n;
    } else {
      return "operator " + ty + " has no counterpart";
    }
    return "";
  };

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
  std::map<int, int> src_linear_by_weight;  // weight root -> kept src pattern node
  int first_src_linear = -1;
  for (size_t i = 0; i < r.src.size(); ++i) {
    if (src.weight_only[i]) continue;
    Conv c;
    e = conv(r.src[i], c);
    if (!e.empty()) return fail(e);
    OperatorPattern op;
    op.type = c.t;
    op.attrs = c.cons;
    std::vector<PatternValue> ins;
    for (size_t k = 0; k < r.src[i].inputs.size(); ++k) {
      if (c.t == OpType::LINEAR && k == 1) continue;
      auto const& t = r.src[i].inputs[k];
      ins.push_back(t.op_id < 0 ? PatternValue::input(pin(t.op_id)) : PatternValue{src.remap.at(t.op_id), t.ts_id});
    }
    int id = s.pattern.add_node(op, ins);
    s.pattern.nodes.back().num_outputs = c.num_outputs;
    if (c.t == OpType::LINEAR) {
      if (first_src_linear < 0) first_src_linear = id;
      src_linear_by_weight.emplace(weight_root(r.src, static_cast<int>(i)), id);
    }
  }
  for (size_t i = 0; i < r.dst.size(); ++i) {
    if (dst.weight_only[i]) continue;
    Conv c;
    e = conv(r.dst[i], c);
    if (!e.empty()) return fail(e);
    OutputOperator o;
    if (c.t == OpType::LINEAR) {
      // out_channels / bias / initializers come from the matched Linear
      // that uses the same weight
      auto it = src_linear_by_weight.find(weight_root(r.dst, static_cast<int>(i)));
      o.copy_from = it != src_linear_by_weight.end() ? it->second : first_src_linear;
      if (o.copy_from < 0) return fail("a Linear with no Linear to take its attributes from");
    } else {
      o.type = c.t;
    }
    for (auto const& kv : c.assign) o.assign.push_back({kv.first, false, -1, "", kv.second});
    for (size_t k = 0; k < r.dst[i].inputs.size(); ++k) {
      if (c.t == OpType::LINEAR && k == 1) continue;
      auto const& t = r.dst[i].inputs[k];
      if (t.op_id < 0) {
        if (!in_index.count(t.op_id)) return fail("output graph reads an input the pattern does not bind");
        o.inputs.push_back(PatternValue::input(in_index.at(t.op_id)));
      } else {
        o.inputs.push_back({dst.remap.at(t.op_id), t.ts_id});
      }
    }
    s.out_nodes.push_back(o);
  }
  for (auto const& m : r.mapped_outputs) {
    if (m.src_op < 0 || m.dst_op < 0 || src.remap.at(m.src_op) < 0 || dst.remap.at(m.dst_op) < 0)
      return fail("mapped output on a weight path");
    s.pattern.outputs.push_back({src.remap.at(m.src_op), m.src_ts});
    s.output_mapping.push_back({dst.remap.at(m.dst_op), m.dst_ts});
  }
  if (s.pattern.nodes.empty()) return fail("empty pattern");
  if (s.pattern.outputs.empty()) return fail("no mapped outputs");
  return s;
}

LegacyRule reverse_legacy_rule(const LegacyRule& r) {
  LegacyRule v;
  v.name = r.name;
  v.src = r.dst;
  v.dst = r.src;
  for (auto const& m : r.mapped_outputs) v.mapped_outputs.push_back({m.dst_op, m.dst_ts, m.src_op, m.src_ts});
  return v;
}

std::vector<Substitution> load_substitutions(const Json& j, std::vector<std::string>* skipped) {
  std::vector<Substitution> out;
  if (j.is_object() && j.contains("rule")) {
    auto coll = load_legacy_rules(j);
    for (auto const& r : coll.rules) {
      std::string why, why_rev;
      auto s = substitution_from_legacy_rule(r, &why);
      if (!s) {
        // a TASO rule states an equivalence: where the left-to-right form
        // cannot be expressed, the right-to-left one may be
        s = substitution_from_legacy_rule(reverse_legacy_rule(r), &why_rev);
        if (s) s->name += "_rev";
      }
      if (s) out.push_back(std::move(*s));
      else if (skipped) skipped->push_back(r.name + ": " + why + " / reversed: " + why_rev);
    }
    return out;
  }
  const Json& arr = j.is_object() ? j.at("substitutions") : j;
  for (auto const& x : arr.as_array()) out.push_back(Substitution::from_json(x));
  return out;
}

std::vector<Substitution> load_substitutions_file(const std::string& path, std::vector<std::string>* skipped) {
  std::ifstream f(path);
  if (!f) throw FFError("cannot read substitution file " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return load_substitutions(Json::parse(ss.str()), skipped);
}

}  // namespace ff
