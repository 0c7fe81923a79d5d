// Graph library: a plain DiGraph with the algorithms the search needs, and a
// labelled dataflow graph (ordered inputs / outputs per node) that backs the
// ComputationGraph and the ParallelComputationGraph.
//
// Parity: lib/utils/include/utils/graph/* (digraph algorithms: topological
// ordering, transitive reduction/closure, dominators, weakly connected
// components, dot export; dataflow graphs with ordered node inputs/outputs).
// Node ids are stable ints (deleted ids are never reused) so that a rewrite
// (substitution) leaves untouched nodes addressable.
#pragma once
#include <algorithm>
#include <queue>
#include <memory>
#include <cstdint>
#include <functional>
#include <map>
#include <optional>
#include <set>
#include <string>
#include <vector>

#include "ff/json.h"
#include "ff/types.h"

namespace ff {

// ---------------------------------------------------------------------------
struct DiGraph {
  std::set<int> nodes;
  std::map<int, std::set<int>> succ, pred;

  void add_node(int n) {
    nodes.insert(n);
    succ[n];
    pred[n];
  }
  void add_edge(int a, int b) {
    add_node(a);
    add_node(b);
    succ[a].insert(b);
    pred[b].insert(a);
  }
  bool has_edge(int a, int b) const {
    auto it = succ.find(a);
    return it != succ.end() && it->second.count(b);
  }
  size_t num_edges() const {
    size_t n = 0;
    for (auto const& kv : succ) n += kv.second.size();
    return n;
  }
  std::vector<int> sources() const;
  std::vector<int> sinks() const;
  DiGraph induced_subgraph(const std::set<int>& keep) const;
};

std::vector<int> topological_order(const DiGraph& g);  // throws on cycle
bool is_acyclic(const DiGraph& g);
// reach[n] = set of nodes reachable from n (excluding n)
std::map<int, std::set<int>> transitive_closure(const DiGraph& g);
DiGraph transitive_reduction(const DiGraph& g);
// dominators[n] = nodes that dominate n (including n), w.r.t. all sources
std::map<int, std::set<int>> dominators(const DiGraph& g);
std::map<int, std::set<int>> post_dominators(const DiGraph& g);
std::vector<std::set<int>> weakly_connected_components(const DiGraph& g);
std::string digraph_as_dot(const DiGraph& g, const std::function<std::string(int)>& label);
// idom[n] = immediate dominator of n (-1 for sources / nodes dominated only by themselves)
std::map<int, int> immediate_dominators(const DiGraph& g);
std::map<int, int> immediate_post_dominators(const DiGraph& g);
// Critical path with node weights: (length, nodes on one longest path).
std::pair<double, std::vector<int>> longest_path(const DiGraph& g, const std::function<double(int)>& weight);
// Graph isomorphism a -> b (node map) respecting node labels (equal strings),
// or nullopt.  Backtracking over a topological order of `a` with degree /
// label / neighbourhood-consistency pruning (DAGs of a few thousand nodes).
std::optional<std::map<int, int>> find_isomorphism(const DiGraph& a, const DiGraph& b,
                                                   const std::function<std::string(int)>& label_a,
                                                   const std::function<std::string(int)>& label_b);
bool is_isomorphic(const DiGraph& a, const DiGraph& b);
// Line digraph L(H): one node per edge of H, e1 -> e2 when head(e1) == tail(e2).
// inverse_line_graph(G) recovers H (nodes = endpoint classes, edge id = node of
// G) if G is a line digraph; nullopt otherwise.
struct InverseLineGraph {
  DiGraph h;                                // endpoint classes as nodes
  std::map<int, std::pair<int, int>> edge;  // node of G -> (tail, head) in h
};
std::optional<InverseLineGraph> inverse_line_graph(const DiGraph& g);

// ---------------------------------------------------------------------------
struct ValueRef {
  int node = -1;
  int idx = 0;
  bool operator==(const ValueRef& o) const { return node == o.node && idx == o.idx; }
  bool operator!=(const ValueRef& o) const { return !(*this == o); }
  bool operator<(const ValueRef& o) const { return node != o.node ? node < o.node : idx < o.idx; }
};

template <typename NodeLabel, typename TensorLabel>
class DataflowGraph {
 public:
  struct Node {
    NodeLabel label;
    std::vector<ValueRef> inputs;
    std::vector<TensorLabel> outputs;
  };

  int add_node(NodeLabel label, std::vector<ValueRef> inputs, std::vector<TensorLabel> outputs) {
    for (auto const& v : inputs) check_value(v);
    int id = next_id_++;
    nodes_[id] = std::make_shared<Node>(Node{std::move(label), std::move(inputs), std::move(outputs)});
    return id;
  }
  // Used by deserialisation / rewrites that must preserve ids.
  void add_node_with_id(int id, NodeLabel label, std::vector<ValueRef> inputs,
                        std::vector<TensorLabel> outputs) {
    if (nodes_.count(id)) throw FFError("duplicate node id " + std::to_string(id));
    nodes_[id] = std::make_shared<Node>(Node{std::move(label), std::move(inputs), std::move(outputs)});
    next_id_ = std::max(next_id_, id + 1);
  }
  void remove_node(int id) { nodes_.erase(id); }
  bool has_node(int id) const { return nodes_.count(id) > 0; }
  const Node& node(int id) const {
    auto it = nodes_.find(id);
    if (it == nodes_.end()) throw FFError("no node " + std::to_string(id));
    return *it->second;
  }
  // Nodes are shared between copies of a graph (a search copies a graph for
  // every candidate rewrite and changes a handful of nodes): mutable access
  // unshares the one node first.
  Node& node(int id) {
    auto it = nodes_.find(id);
    if (it == nodes_.end()) throw FFError("no node " + std::to_string(id));
    return unshare(it->second);
  }
  const TensorLabel& tensor(ValueRef v) const { return node(v.node).outputs.at(v.idx); }
  TensorLabel& tensor(ValueRef v) { return node(v.node).outputs.at(v.idx); }
  std::vector<int> node_ids() const {
    std::vector<int> r;
    r.reserve(nodes_.size());
    for (auto const& kv : nodes_) r.push_back(kv.first);
    return r;
  }
  size_t num_nodes() const { return nodes_.size(); }
  int next_id() const { return next_id_; }

  DiGraph digraph() const {
    DiGraph g;
    for (auto const& kv : nodes_) {
      g.add_node(kv.first);
      for (auto const& v : kv.second->inputs) g.add_edge(v.node, kv.first);
    }
    return g;
  }
  // Kahn's algorithm, smallest ready id first (the order of
  // topological_order(digraph()), without building the DiGraph).
  std::vector<int> topo_order() const {
    const int n = next_id_;
    // distinct predecessors per node, as CSR arrays (no per-node allocation)
    std::vector<int> indeg(n, -1), off(n + 1, 0), edges_from, edges_to;
    edges_from.reserve(nodes_.size() * 2);
    edges_to.reserve(nodes_.size() * 2);
    int preds[64];
    for (auto const& kv : nodes_) {
      auto const& in = kv.second->inputs;
      int k = 0;
      std::vector<int> big;
      int* pp = preds;
      if (in.size() > 64) {
        big.resize(in.size());
        pp = big.data();
      }
      for (auto const& v : in) pp[k++] = v.node;
      std::sort(pp, pp + k);
      k = static_cast<int>(std::unique(pp, pp + k) - pp);
      indeg[kv.first] = k;
      for (int i = 0; i < k; ++i) {
        int p = pp[i];
        if (p < 0 || p >= n || !nodes_.count(p)) throw FFError("dangling value reference " + std::to_string(p));
        edges_from.push_back(p);
        edges_to.push_back(kv.first);
        ++off[p + 1];
      }
    }
    for (int i = 0; i < n; ++i) off[i + 1] += off[i];
    std::vector<int> succ(edges_to.size()), fill(off.begin(), off.end() - 1);
    for (size_t e = 0; e < edges_to.size(); ++e) succ[fill[edges_from[e]]++] = edges_to[e];
    std::priority_queue<int, std::vector<int>, std::greater<int>> q;
    for (auto const& kv : nodes_)
      if (indeg[kv.first] == 0) q.push(kv.first);
    std::vector<int> order;
    order.reserve(nodes_.size());
    while (!q.empty()) {
      int x = q.top();
      q.pop();
      order.push_back(x);
      for (int e = off[x]; e < off[x + 1]; ++e)
        if (--indeg[succ[e]] == 0) q.push(succ[e]);
    }
    if (order.size() != nodes_.size()) throw FFError("graph has a cycle");
    return order;
  }

  // All (consumer node, input slot) pairs reading value v.
  std::vector<std::pair<int, int>> uses(ValueRef v) const {
    std::vector<std::pair<int, int>> r;
    for (auto const& kv : nodes_)
      for (size_t i = 0; i < kv.second->inputs.size(); ++i)
        if (kv.second->inputs[i] == v) r.push_back({kv.first, static_cast<int>(i)});
    return r;
  }
  std::vector<ValueRef> all_values() const {
    std::vector<ValueRef> r;
    for (auto const& kv : nodes_)
      for (size_t i = 0; i < kv.second->outputs.size(); ++i) r.push_back({kv.first, static_cast<int>(i)});
    return r;
  }
  void replace_uses(ValueRef from, ValueRef to) {
    for (auto& kv : nodes_) {
      bool hit = false;
      for (auto const& v : kv.second->inputs) hit = hit || v == from;
      if (!hit) continue;
      for (auto& v : unshare(kv.second).inputs)
        if (v == from) v = to;
    }
  }

 private:
  static Node& unshare(std::shared_ptr<Node>& p) {
    if (p.use_count() > 1) p = std::make_shared<Node>(*p);
    return *p;
  }
  void check_value(const ValueRef& v) const {
    auto it = nodes_.find(v.node);
    if (it == nodes_.end() || v.idx < 0 || v.idx >= static_cast<int>(it->second->outputs.size()))
      throw FFError("dangling value reference " + std::to_string(v.node) + ":" + std::to_string(v.idx));
  }
  std::map<int, std::shared_ptr<Node>> nodes_;
  int next_id_ = 0;
};

}  // namespace ff
