#include "ff/sp.h"

#include <algorithm>
#include <functional>
#include <cstdint>
#include <map>

namespace ff {

namespace {

using Bits = std::vector<uint64_t>;

struct Ctx {
  std::vector<int> ids;            // index -> node id (global topological order)
  std::map<int, int> index;        // node id -> index
  std::vector<Bits> reach;         // strict descendants
  std::vector<std::vector<int>> succ, pred;
  size_t W = 0;
  bool relaxed = false;
  bool failed = false;
  SPTree tree;
};

inline bool test(const Bits& b, int i) { return (b[i >> 6] >> (i & 63)) & 1; }
inline void set(Bits& b, int i) { b[i >> 6] |= uint64_t(1) << (i & 63); }

// nodes: indices in topological order
int build(Ctx& c, const std::vector<int>& nodes);

std::vector<std::vector<int>> components(Ctx& c, const std::vector<int>& nodes) {
  std::map<int, int> pos;
  for (size_t i = 0; i < nodes.size(); ++i) pos[nodes[i]] = static_cast<int>(i);
  std::vector<int> parent(nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) parent[i] = static_cast<int>(i);
  std::function<int(int)> find = [&](int x) { return parent[x] == x ? x : parent[x] = find(parent[x]); };
  for (size_t i = 0; i < nodes.size(); ++i)
    for (int s : c.succ[nodes[i]]) {
      auto it = pos.find(s);
      if (it != pos.end()) parent[find(static_cast<int>(i))] = find(it->second);
    }
  std::map<int, std::vector<int>> groups;
  for (size_t i = 0; i < nodes.size(); ++i) groups[find(static_cast<int>(i))].push_back(nodes[i]);
  std::vector<std::vector<int>> out;
  for (auto& kv : groups) out.push_back(kv.second);
  std::sort(out.begin(), out.end(), [](auto const& a, auto const& b) { return a.front() < b.front(); });
  return out;
}

int fold(Ctx& c, SPTree::Kind k, const std::vector<int>& parts, bool relaxed = false) {
  int acc = parts.back();
  for (int i = static_cast<int>(parts.size()) - 2; i >= 0; --i) acc = c.tree.add_split(k, parts[i], acc, relaxed);
  return acc;
}

int build(Ctx& c, const std::vector<int>& nodes) {
  if (nodes.size() == 1) return c.tree.add_leaf(c.ids[nodes[0]]);
  auto comps = components(c, nodes);
  if (comps.size() > 1) {
    std::vector<int> parts;
    for (auto const& comp : comps) parts.push_back(build(c, comp));
    return fold(c, SPTree::PARALLEL, parts);
  }
  // series split points: prefix [0,k) all reach suffix [k,n)
  const size_t n = nodes.size();
  Bits inter(c.W, ~uint64_t(0));
  Bits suffix(c.W, 0);
  std::vector<Bits> suf(n + 1, Bits(c.W, 0));
  for (size_t k = n; k-- > 0;) {
    suf[k] = suf[k + 1];
    set(suf[k], nodes[k]);
  }
  std::vector<size_t> cuts;
  for (size_t k = 1; k < n; ++k) {
    auto const& r = c.reach[nodes[k - 1]];
    for (size_t w = 0; w < c.W; ++w) inter[w] &= r[w];
    bool ok = true;
    for (size_t w = 0; w < c.W && ok; ++w)
      if ((suf[k][w] & ~inter[w]) != 0) ok = false;
    if (ok) cuts.push_back(k);
  }
  if (!cuts.empty()) {
    std::vector<int> parts;
    size_t lo = 0;
    cuts.push_back(n);
    for (size_t k : cuts) {
      parts.push_back(build(c, std::vector<int>(nodes.begin() + lo, nodes.begin() + k)));
      lo = k;
    }
    return fold(c, SPTree::SERIES, parts);
  }
  if (!c.relaxed) {
    c.failed = true;
    return c.tree.add_leaf(c.ids[nodes[0]]);
  }
  // relaxed: cut with the fewest crossing edges (ties -> closest to middle)
  std::map<int, int> pos;
  for (size_t i = 0; i < n; ++i) pos[nodes[i]] = static_cast<int>(i);
  std::vector<int> delta(n + 1, 0);  // crossing(k) = #edges (i<k<=j)
  for (size_t i = 0; i < n; ++i)
    for (int s : c.succ[nodes[i]]) {
      auto it = pos.find(s);
      if (it == pos.end()) continue;
      delta[i + 1] += 1;
      delta[it->second + 1] -= 1;
    }
  int best_k = 1;
  long best = -1;
  int run = 0;
  for (size_t k = 1; k < n; ++k) {
    run += delta[k];
    long score = static_cast<long>(run) * static_cast<long>(4 * n) +
                 std::labs(static_cast<long>(2 * k) - static_cast<long>(n));
    if (best < 0 || score < best) {
      best = score;
      best_k = static_cast<int>(k);
    }
  }
  int l = build(c, std::vector<int>(nodes.begin(), nodes.begin() + best_k));
  int r = build(c, std::vector<int>(nodes.begin() + best_k, nodes.end()));
  return c.tree.add_split(SPTree::SERIES, l, r, true);
}

Ctx make_ctx(const DiGraph& g, bool relaxed) {
  Ctx c;
  c.relaxed = relaxed;
  c.ids = topological_order(g);
  for (size_t i = 0; i < c.ids.size(); ++i) c.index[c.ids[i]] = static_cast<int>(i);
  const size_t n = c.ids.size();
  c.W = (n + 63) / 64;
  c.succ.assign(n, {});
  c.pred.assign(n, {});
  for (size_t i = 0; i < n; ++i) {
    auto it = g.succ.find(c.ids[i]);
    if (it == g.succ.end()) continue;
    for (int s : it->second) {
      c.succ[i].push_back(c.index.at(s));
      c.pred[c.index.at(s)].push_back(static_cast<int>(i));
    }
  }
  c.reach.assign(n, Bits(c.W, 0));
  for (size_t i = n; i-- > 0;)
    for (int s : c.succ[i]) {
      set(c.reach[i], s);
      for (size_t w = 0; w < c.W; ++w) c.reach[i][w] |= c.reach[s][w];
    }
  return c;
}

}  // namespace

std::vector<int> SPTree::leaves(int idx) const {
  std::vector<int> out;
  std::vector<int> st{idx};
  while (!st.empty()) {
    int i = st.back();
    st.pop_back();
    auto const& x = e.at(i);
    if (x.kind == LEAF) out.push_back(x.node);
    else {
      st.push_back(x.right);
      st.push_back(x.left);
    }
  }
  return out;
}

int SPTree::num_relaxed() const {
  int n = 0;
  for (auto const& x : e) n += x.relaxed ? 1 : 0;
  return n;
}

Json SPTree::to_json(int idx) const {
  auto const& x = e.at(idx);
  if (x.kind == LEAF) return Json(x.node);
  Json ch = Json::array();
  std::vector<int> st{idx};
  // flatten same-kind chains into an n-ary node
  std::function<void(int)> collect = [&](int i) {
    auto const& y = e.at(i);
    if (y.kind == x.kind && !y.relaxed == !x.relaxed) {
      collect(y.left);
      collect(y.right);
    } else {
      ch.push_back(to_json(i));
    }
  };
  collect(x.left);
  collect(x.right);
  Json j = Json::object();
  j["type"] = x.kind == SERIES ? (x.relaxed ? "series_relaxed" : "series") : "parallel";
  j["children"] = ch;
  return j;
}

Json SPTree::to_json() const { return root < 0 ? Json() : to_json(root); }

std::optional<SPTree> get_series_parallel_decomposition(const DiGraph& g) {
  if (g.nodes.empty()) return std::nullopt;
  Ctx c = make_ctx(g, false);
  std::vector<int> all(c.ids.size());
  for (size_t i = 0; i < all.size(); ++i) all[i] = static_cast<int>(i);
  c.tree.root = build(c, all);
  if (c.failed) return std::nullopt;
  return c.tree;
}

SPTree get_relaxed_sp_decomposition(const DiGraph& g) {
  if (g.nodes.empty()) return SPTree{};
  Ctx c = make_ctx(g, true);
  std::vector<int> all(c.ids.size());
  for (size_t i = 0; i < all.size(); ++i) all[i] = static_cast<int>(i);
  c.tree.root = build(c, all);
  return c.tree;
}

bool is_series_parallel(const DiGraph& g) { return get_series_parallel_decomposition(g).has_value(); }

// ---------------------------------------------------------------------------
std::vector<BinaryTreePath> find_paths_to_leaf(const SPTree& t, int node) {
  std::vector<BinaryTreePath> out;
  BinaryTreePath cur;
  std::function<void(int)> rec = [&](int i) {
    if (i < 0) return;
    const auto& e = t.e[i];
    if (e.kind == SPTree::LEAF) {
      if (e.node == node) out.push_back(cur);
      return;
    }
    cur.push_back(0);
    rec(e.left);
    cur.back() = 1;
    rec(e.right);
    cur.pop_back();
  };
  rec(t.root);
  return out;
}

int get_subtree_at_path(const SPTree& t, const BinaryTreePath& path) {
  int i = t.root;
  for (int step : path) {
    if (i < 0 || t.e[i].kind == SPTree::LEAF) return -1;
    i = step == 0 ? t.e[i].left : t.e[i].right;
  }
  return i;
}

static SPTree reassociate(const SPTree& t, bool left) {
  SPTree r;
  // flatten maximal chains of the same split kind (relaxed series cuts are kept
  // as chain boundaries: they carry their own cost semantics)
  std::function<void(int, SPTree::Kind, std::vector<int>&)> flatten = [&](int i, SPTree::Kind k,
                                                                          std::vector<int>& items) {
    const auto& e = t.e[i];
    if (e.kind == k && !e.relaxed) {
      flatten(e.left, k, items);
      flatten(e.right, k, items);
    } else {
      items.push_back(i);
    }
  };
  std::function<int(int)> build = [&](int i) -> int {
    const auto& e = t.e[i];
    if (e.kind == SPTree::LEAF) return r.add_leaf(e.node);
    if (e.relaxed) return r.add_split(e.kind, build(e.left), build(e.right), true);
    std::vector<int> items;
    flatten(i, e.kind, items);
    std::vector<int> built;
    for (int it : items) built.push_back(build(it));
    if (left) {
      int acc = built[0];
      for (size_t j = 1; j < built.size(); ++j) acc = r.add_split(e.kind, acc, built[j]);
      return acc;
    }
    int acc = built.back();
    for (size_t j = built.size() - 1; j-- > 0;) acc = r.add_split(e.kind, built[j], acc);
    return acc;
  };
  if (t.root >= 0) r.root = build(t.root);
  return r;
}
SPTree left_associative(const SPTree& t) { return reassociate(t, true); }
SPTree right_associative(const SPTree& t) { return reassociate(t, false); }

}  // namespace ff
