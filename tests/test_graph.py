"""Graph library (csrc/ffcore/src/graph.cc, sp.cc) — parity with the
reference's lib/utils/test/src/utils/graph/** cases: topological order,
transitive closure / reduction, (immediate) dominators, weakly connected
components, isomorphism, inverse line graph, critical path, and the binary SP
tree path utilities (utils/full_binary_tree)."""
import itertools
import random

import pytest

from flexflow_train_amd import _ffcore as C

G = C.graph

# diamond with a tail: 0 -> {1, 2} -> 3 -> 4, plus a transitive edge 0 -> 3
N = [0, 1, 2, 3, 4]
E = [(0, 1), (0, 2), (1, 3), (2, 3), (3, 4), (0, 3)]


def test_topo_and_cycle():
    order = G.topological_order(N, E)
    pos = {n: i for i, n in enumerate(order)}
    assert all(pos[a] < pos[b] for a, b in E)
    assert G.is_acyclic(N, E)
    assert not G.is_acyclic([0, 1], [(0, 1), (1, 0)])
    with pytest.raises(ValueError):
        G.topological_order([0, 1], [(0, 1), (1, 0)])


def test_closure_and_reduction():
    clo = set(G.transitive_closure(N, E))
    assert (0, 4) in clo and (1, 4) in clo and (4, 0) not in clo
    red = set(G.transitive_reduction(N, E))
    assert red == {(0, 1), (0, 2), (1, 3), (2, 3), (3, 4)}
    # reduction preserves reachability
    assert set(G.transitive_closure(N, list(red))) == clo


def test_dominators():
    dom = G.dominators(N, E)
    assert dom[3] == {0, 3} and dom[4] == {0, 3, 4} and dom[1] == {0, 1}
    idom = G.immediate_dominators(N, E)
    assert idom[0] == -1 and idom[1] == 0 and idom[3] == 0 and idom[4] == 3
    ipdom = G.immediate_post_dominators(N, E)
    assert ipdom[1] == 3 and ipdom[0] == 3 and ipdom[4] == -1


def test_weak_components_and_longest_path():
    comps = G.weakly_connected_components([0, 1, 2, 3, 9], [(0, 1), (2, 3)])
    assert sorted(sorted(c) for c in comps) == [[0, 1], [2, 3], [9]]
    length, path = G.longest_path(N, E, {0: 1.0, 1: 5.0, 2: 1.0, 3: 1.0, 4: 2.0})
    assert length == 9.0 and path == [0, 1, 3, 4]


def _relabel(nodes, edges, perm):
    return [perm[n] for n in nodes], [(perm[a], perm[b]) for a, b in edges]


def test_isomorphism_random_dags():
    rng = random.Random(0)
    for trial in range(20):
        n = rng.randint(3, 12)
        nodes = list(range(n))
        edges = [(a, b) for a, b in itertools.combinations(nodes, 2) if rng.random() < 0.3]
        perm = dict(zip(nodes, rng.sample(range(100, 100 + n), n)))
        nb, eb = _relabel(nodes, edges, perm)
        m = G.find_isomorphism(nodes, edges, nb, eb)
        assert m is not None
        assert {(m[a], m[b]) for a, b in edges} == set(eb)
        if edges:  # dropping an edge breaks it
            assert G.find_isomorphism(nodes, edges, nb, eb[1:]) is None


def test_isomorphism_respects_labels():
    nodes, edges = [0, 1, 2], [(0, 1), (0, 2)]
    la = {0: "in", 1: "relu", 2: "linear"}
    assert G.find_isomorphism(nodes, edges, [5, 6, 7], [(5, 6), (5, 7)], la,
                              {5: "in", 6: "linear", 7: "relu"}) == {0: 5, 1: 7, 2: 6}
    assert G.find_isomorphism(nodes, edges, [5, 6, 7], [(5, 6), (5, 7)], la,
                              {5: "in", 6: "linear", 7: "linear"}) is None


def _line_graph(h_edges):
    """nodes = edge ids of H, e1 -> e2 when head(e1) == tail(e2)."""
    ids = list(range(len(h_edges)))
    return ids, [(i, j) for i in ids for j in ids if h_edges[i][1] == h_edges[j][0]]


def test_inverse_line_graph_roundtrip():
    # H: a small series-parallel multigraph s -> {a, b} -> t, parallel edges a => t
    h = [(0, 1), (0, 2), (1, 3), (1, 3), (2, 3), (3, 4)]
    nodes, edges = _line_graph(h)
    r = G.inverse_line_graph(nodes, edges)
    assert r is not None
    hn, he, emap = r
    assert len(hn) == 5 and len(emap) == len(h)
    # L(recovered H) == G
    rec = [emap[i] for i in nodes]
    assert set(_line_graph(rec)[1]) == set(edges)
    # a digraph that is not a line digraph: succ(0) and succ(1) overlap but differ
    assert G.inverse_line_graph([0, 1, 2, 3], [(0, 2), (1, 2), (1, 3)]) is None


def test_sp_tree_paths_and_associativity():
    # series chain 0 -> 1 -> 2 -> 3
    nodes, edges = [0, 1, 2, 3], [(0, 1), (1, 2), (2, 3)]
    left = G.sp_associative(nodes, edges, True)
    right = G.sp_associative(nodes, edges, False)
    assert left == ("S", ("S", ("S", 0, 1), 2), 3)
    assert right == ("S", 0, ("S", 1, ("S", 2, 3)))
    for n in nodes:
        paths = G.sp_paths_to_leaf(nodes, edges, n)
        assert len(paths) == 1
        assert G.sp_subtree_leaves_at_path(nodes, edges, paths[0]) == [n]
    assert G.sp_subtree_leaves_at_path(nodes, edges, []) == [0, 1, 2, 3]
    # parallel branches
    pn, pe = [0, 1, 2, 3], [(0, 1), (0, 2), (1, 3), (2, 3)]
    assert sorted(G.sp_subtree_leaves_at_path(pn, pe, [])) == [0, 1, 2, 3]
    assert G.sp_subtree_leaves_at_path(pn, pe, [0, 0, 0, 0, 0, 0]) is None


def test_dot_export():
    dot = G.as_dot(N, E)
    assert dot.startswith("digraph") and "->" in dot


# ---- get_series_parallel_decomposition, the reference's cases
# (lib/utils/test/src/utils/graph/series_parallel/get_series_parallel_decomposition.cc)
def _nary(t):
    """binary ("S"|"P", l, r) tree -> n-ary normal form: series = tuple of
    children in order, parallel = frozenset, nested same-kind splits flattened"""
    if isinstance(t, int):
        return t
    kind, l, r = t
    kids = []
    for c in (l, r):
        c = _nary(c)
        same = (kind == "S" and isinstance(c, tuple) and c[0] == "S") or (kind == "P" and isinstance(c, frozenset))
        if same:
            kids.extend(c[1:] if kind == "S" else c)
        else:
            kids.append(c)
    return ("S", *kids) if kind == "S" else frozenset(kids)


def S(*k):
    return ("S", *k)


def P(*k):
    return frozenset(k)


@pytest.mark.parametrize("nodes,edges,want", [
    ([0], [], 0),                                                                  # base case
    ([0, 1], [], P(0, 1)),                                                         # parallel
    ([0, 1], [(0, 1)], S(0, 1)),                                                   # serial
    ([0, 1, 2], [(0, 1), (0, 2)], S(0, P(1, 2))),                                  # composite
    ([0, 1, 2, 3, 4, 5], [(0, 1), (0, 2), (1, 3), (2, 4), (3, 5), (4, 5)],
     S(0, P(S(1, 3), S(2, 4)), 5)),                                                # diamond
    ([0, 1, 2, 3], [(0, 2), (0, 3), (1, 2), (1, 3)], S(P(0, 1), P(2, 3))),        # all-to-all
    ([0, 1, 2, 3], [(0, 2), (1, 2), (1, 3)], None),                                # N graph: not SP
    ([0, 1, 2, 3], [(0, 1), (0, 2), (1, 2), (1, 3), (2, 3)], S(0, 1, 2, 3)),      # needs transitive reduction
], ids=["base", "parallel", "serial", "composite", "diamond", "all_to_all", "non_sp", "transitive"])
def test_series_parallel_decomposition_reference(nodes, edges, want):
    t = G.sp_decomposition(nodes, edges)
    assert (None if t is None else _nary(t)) == want
