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

}  // namespace ff
