// Series-parallel decomposition of a DAG.
//
// Parity: utils/graph/series_parallel/get_series_parallel_decomposition.cc
// (sp.cc:18-93) and compiler/series_parallel/computation_graph/* (plain SP
// first; fall back by adding edges from sources).  The reference reduces the
// inverse line graph; here we decompose directly on the transitive closure
// (bitsets): a top-level series split point is a topological cut where every
// node before it reaches every node after it, a parallel split is a weakly
// connected component split.  All series split points of a level are taken
// at once, so the decomposition is O(n^2/64) per nesting level.
//
// `get_relaxed_sp_decomposition` never fails: where neither split exists it
// cuts the topological order at the point with the fewest crossing edges and
// marks the series node `relaxed` — used by the machine-mapping DP on
// non-SP PCGs (skip connections crossing attention blocks, shared weights).
#pragma once
#include <optional>
#include <vector>

#include "ff/graph.h"
#include "ff/json.h"

namespace ff {

struct SPTree {
  enum Kind { LEAF = 0, SERIES = 1, PARALLEL = 2 };
  struct Entry {
    Kind kind = LEAF;
    int node = -1;  // LEAF only
    int left = -1, right = -1;
    bool relaxed = false;
  };
  std::vector<Entry> e;
  int root = -1;

  int add_leaf(int node) {
    e.push_back({LEAF, node, -1, -1, false});
    return static_cast<int>(e.size()) - 1;
  }
  int add_split(Kind k, int l, int r, bool relaxed = false) {
    e.push_back({k, -1, l, r, relaxed});
    return static_cast<int>(e.size()) - 1;
  }
  std::vector<int> leaves(int idx) const;
  std::vector<int> leaves() const { return root < 0 ? std::vector<int>{} : leaves(root); }
  int num_relaxed() const;
  // Nested n-ary JSON: {"type": "series"|"parallel", "children": [...]} / node id.
  Json to_json() const;
  Json to_json(int idx) const;
};

// Paths in the binary tree (parity: utils/full_binary_tree/binary_tree_path,
// find_paths_to_leaf, get_subtree_at_path — machine-mapping results are keyed
// by path).  A path is a sequence of 0 (left) / 1 (right) from the root.
using BinaryTreePath = std::vector<int>;
std::vector<BinaryTreePath> find_paths_to_leaf(const SPTree& t, int node);
int get_subtree_at_path(const SPTree& t, const BinaryTreePath& path);  // entry index, -1 if invalid
// Re-associate maximal same-kind chains left-deep (((a b) c) d) or right-deep.
SPTree left_associative(const SPTree& t);
SPTree right_associative(const SPTree& t);

std::optional<SPTree> get_series_parallel_decomposition(const DiGraph& g);
SPTree get_relaxed_sp_decomposition(const DiGraph& g);
bool is_series_parallel(const DiGraph& g);

}  // namespace ff
