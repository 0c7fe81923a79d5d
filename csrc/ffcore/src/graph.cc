#include "ff/graph.h"

#include <algorithm>
#include <deque>
#include <queue>
#include <sstream>

namespace ff {

std::vector<int> DiGraph::sources() const {
  std::vector<int> r;
  for (int n : nodes)
    if (pred.at(n).empty()) r.push_back(n);
  return r;
}

std::vector<int> DiGraph::sinks() const {
  std::vector<int> r;
  for (int n : nodes)
    if (succ.at(n).empty()) r.push_back(n);
  return r;
}

DiGraph DiGraph::induced_subgraph(const std::set<int>& keep) const {
  DiGraph g;
  for (int n : keep) {
    if (!nodes.count(n)) continue;
    g.add_node(n);
  }
  for (int n : keep) {
    if (!nodes.count(n)) continue;
    for (int s : succ.at(n))
      if (keep.count(s)) g.add_edge(n, s);
  }
  return g;
}

std::vector<int> topological_order(const DiGraph& g) {
  std::map<int, int> indeg;
  for (int n : g.nodes) indeg[n] = static_cast<int>(g.pred.at(n).size());
  // min-heap on node id -> deterministic order
  std::priority_queue<int, std::vector<int>, std::greater<int>> q;
  for (auto const& kv : indeg)
    if (kv.second == 0) q.push(kv.first);
  std::vector<int> order;
  while (!q.empty()) {
    int n = q.top();
    q.pop();
    order.push_back(n);
    for (int s : g.succ.at(n))
      if (--indeg[s] == 0) q.push(s);
  }
  if (order.size() != g.nodes.size()) throw FFError("graph has a cycle");
  return order;
}

bool is_acyclic(const DiGraph& g) {
  try {
    topological_order(g);
    return true;
  } catch (FFError const&) {
    return false;
  }
}

std::map<int, std::set<int>> transitive_closure(const DiGraph& g) {
  auto order = topological_order(g);
  std::map<int, std::set<int>> reach;
  for (auto it = order.rbegin(); it != order.rend(); ++it) {
    auto& r = reach[*it];
    for (int s : g.succ.at(*it)) {
      r.insert(s);
      auto const& rs = reach[s];
      r.insert(rs.begin(), rs.end());
    }
  }
  return reach;
}

DiGraph transitive_reduction(const DiGraph& g) {
  auto reach = transitive_closure(g);
  DiGraph r;
  for (int n : g.nodes) r.add_node(n);
  for (int a : g.nodes) {
    for (int b : g.succ.at(a)) {
      bool redundant = false;
      for (int c : g.succ.at(a)) {
        if (c != b && reach[c].count(b)) {
          redundant = true;
          break;
        }
      }
      if (!redundant) r.add_edge(a, b);
    }
  }
  return r;
}

static std::map<int, std::set<int>> dominators_impl(const DiGraph& g, bool post) {
  auto order = topological_order(g);
  if (post) std::reverse(order.begin(), order.end());
  auto const& preds = post ? g.succ : g.pred;
  std::map<int, std::set<int>> dom;
  for (int n : order) {
    auto const& ps = preds.at(n);
    std::set<int> d;
    bool first = true;
    for (int p : ps) {
      if (first) {
        d = dom[p];
        first = false;
      } else {
        std::set<int> tmp;
        std::set_intersection(d.begin(), d.end(), dom[p].begin(), dom[p].end(),
                              std::inserter(tmp, tmp.begin()));
        d.swap(tmp);
      }
    }
    d.insert(n);
    dom[n] = std::move(d);
  }
  return dom;
}

std::map<int, std::set<int>> dominators(const DiGraph& g) { return dominators_impl(g, false); }
std::map<int, std::set<int>> post_dominators(const DiGraph& g) { return dominators_impl(g, true); }

std::vector<std::set<int>> weakly_connected_components(const DiGraph& g) {
  std::set<int> seen;
  std::vector<std::set<int>> comps;
  for (int n : g.nodes) {
    if (seen.count(n)) continue;
    std::set<int> comp;
    std::deque<int> q{n};
    seen.insert(n);
    while (!q.empty()) {
      int x = q.front();
      q.pop_front();
      comp.insert(x);
      for (int y : g.succ.at(x))
        if (seen.insert(y).second) q.push_back(y);
      for (int y : g.pred.at(x))
        if (seen.insert(y).second) q.push_back(y);
    }
    comps.push_back(std::move(comp));
  }
  return comps;
}

std::string digraph_as_dot(const DiGraph& g, const std::function<std::string(int)>& label) {
  std::ostringstream os;
  os << "digraph G {\n";
  for (int n : g.nodes) {
    std::string l = label ? label(n) : std::to_string(n);
    std::string esc;
    for (char c : l) {
      if (c == '"') esc += "\\\"";
      else esc.push_back(c);
    }
    os << "  n" << n << " [label=\"" << esc << "\"];\n";
  }
  for (int a : g.nodes)
    for (int b : g.succ.at(a)) os << "  n" << a << " -> n" << b << ";\n";
  os << "}\n";
  return os.str();
}

// ---------------------------------------------------------------------------
static std::map<int, int> idom_impl(const DiGraph& g, bool post) {
  auto dom = post ? post_dominators(g) : dominators(g);
  std::map<int, int> idom;
  for (auto const& kv : dom) {
    // the strict dominator with the largest dominator set is the immediate one
    int best = -1;
    size_t best_sz = 0;
    for (int d : kv.second) {
      if (d == kv.first) continue;
      const size_t sz = dom[d].size();
      if (best < 0 || sz > best_sz) {
        best = d;
        best_sz = sz;
      }
    }
    idom[kv.first] = best;
  }
  return idom;
}
std::map<int, int> immediate_dominators(const DiGraph& g) { return idom_impl(g, false); }
std::map<int, int> immediate_post_dominators(const DiGraph& g) { return idom_impl(g, true); }

std::pair<double, std::vector<int>> longest_path(const DiGraph& g, const std::function<double(int)>& weight) {
  auto order = topological_order(g);
  std::map<int, double> dist;
  std::map<int, int> from;
  double best = 0.0;
  int end = -1;
  for (int n : order) {
    double d = 0.0;
    int f = -1;
    for (int p : g.pred.at(n))
      if (f < 0 || dist[p] > d) {
        d = dist[p];
        f = p;
      }
    dist[n] = d + weight(n);
    from[n] = f;
    if (end < 0 || dist[n] > best) {
      best = dist[n];
      end = n;
    }
  }
  std::vector<int> path;
  for (int n = end; n >= 0; n = from[n]) path.push_back(n);
  std::reverse(path.begin(), path.end());
  return {best, path};
}

std::optional<std::map<int, int>> find_isomorphism(const DiGraph& a, const DiGraph& b,
                                                   const std::function<std::string(int)>& label_a,
                                                   const std::function<std::string(int)>& label_b) {
  if (a.nodes.size() != b.nodes.size() || a.num_edges() != b.num_edges()) return std::nullopt;
  // invariant signature per node: (label, in-degree, out-degree)
  auto sig = [](const DiGraph& g, int n, const std::function<std::string(int)>& lab) {
    return lab(n) + "#" + std::to_string(g.pred.at(n).size()) + "#" + std::to_string(g.succ.at(n).size());
  };
  std::map<std::string, std::vector<int>> cand_b;
  std::map<std::string, int> count_a;
  for (int n : b.nodes) cand_b[sig(b, n, label_b)].push_back(n);
  for (int n : a.nodes) count_a[sig(a, n, label_a)]++;
  for (auto const& kv : count_a) {
    auto it = cand_b.find(kv.first);
    if (it == cand_b.end() || static_cast<int>(it->second.size()) != kv.second) return std::nullopt;
  }
  std::vector<int> order;
  try {
    order = topological_order(a);
  } catch (FFError const&) {
    order.assign(a.nodes.begin(), a.nodes.end());
  }
  std::vector<std::string> sigs;
  for (int n : order) sigs.push_back(sig(a, n, label_a));
  std::map<int, int> fwd, bwd;
  long budget = 2000000;  // backtracking step cap (adversarial regular graphs)
  std::function<bool(size_t)> rec = [&](size_t i) -> bool {
    if (i == order.size()) return true;
    if (--budget < 0) return false;
    const int u = order[i];
    for (int v : cand_b[sigs[i]]) {
      if (bwd.count(v)) continue;
      bool ok = true;
      // every already-mapped neighbour of u must map to the matching neighbour of v
      for (int p : a.pred.at(u))
        if (fwd.count(p) && !b.has_edge(fwd[p], v)) { ok = false; break; }
      if (ok)
        for (int s : a.succ.at(u))
          if (fwd.count(s) && !b.has_edge(v, fwd[s])) { ok = false; break; }
      if (ok) {  // and vice versa (edges of v into mapped nodes exist in a)
        for (int p : b.pred.at(v))
          if (bwd.count(p) && !a.has_edge(bwd[p], u)) { ok = false; break; }
        if (ok)
          for (int s : b.succ.at(v))
            if (bwd.count(s) && !a.has_edge(u, bwd[s])) { ok = false; break; }
      }
      if (!ok) continue;
      fwd[u] = v;
      bwd[v] = u;
      if (rec(i + 1)) return true;
      fwd.erase(u);
      bwd.erase(v);
    }
    return false;
  };
  if (!rec(0)) return std::nullopt;
  return fwd;
}

bool is_isomorphic(const DiGraph& a, const DiGraph& b) {
  auto none = [](int) { return std::string(); };
  return find_isomorphism(a, b, none, none).has_value();
}

std::optional<InverseLineGraph> inverse_line_graph(const DiGraph& g) {
  // endpoints: tail(v) = 2*i, head(v) = 2*i+1; an edge u -> w of G glues head(u) to tail(w)
  std::vector<int> ids(g.nodes.begin(), g.nodes.end());
  std::map<int, int> idx;
  for (size_t i = 0; i < ids.size(); ++i) idx[ids[i]] = static_cast<int>(i);
  std::vector<int> parent(2 * ids.size());
  for (size_t i = 0; i < parent.size(); ++i) parent[i] = static_cast<int>(i);
  std::function<int(int)> find = [&](int x) { return parent[x] == x ? x : parent[x] = find(parent[x]); };
  auto unite = [&](int a, int c) {
    a = find(a);
    c = find(c);
    if (a != c) parent[a] = c;
  };
  for (int u : ids)
    for (int w : g.succ.at(u)) unite(2 * idx[u] + 1, 2 * idx[w]);
  // one source node (all tails of predecessor-less edges) and one sink node
  // (all heads of successor-less edges), the convention of the SP reduction
  int src = -1, snk = -1;
  for (int v : ids) {
    if (g.pred.at(v).empty()) {
      if (src >= 0) unite(src, 2 * idx[v]);
      src = 2 * idx[v];
    }
    if (g.succ.at(v).empty()) {
      if (snk >= 0) unite(snk, 2 * idx[v] + 1);
      snk = 2 * idx[v] + 1;
    }
  }
  // line-digraph check: u -> w in G  <=>  head(u) ~ tail(w)
  std::map<int, std::vector<int>> by_tail;
  for (int w : ids) by_tail[find(2 * idx[w])].push_back(w);
  for (int u : ids) {
    const auto it = by_tail.find(find(2 * idx[u] + 1));
    const size_t n_glued = it == by_tail.end() ? 0 : it->second.size();
    if (n_glued != g.succ.at(u).size()) return std::nullopt;
  }
  InverseLineGraph r;
  std::map<int, int> cls;
  auto node_of = [&](int end) {
    const int c = find(end);
    auto it = cls.find(c);
    if (it != cls.end()) return it->second;
    const int id = static_cast<int>(cls.size());
    cls[c] = id;
    r.h.add_node(id);
    return id;
  };
  for (int v : ids) {
    const int t = node_of(2 * idx[v]), h = node_of(2 * idx[v] + 1);
    r.edge[v] = {t, h};
    r.h.add_edge(t, h);
  }
  return r;
}

}  // namespace ff
