"""MachineView -> machine coordinate semantics, the cases of the reference's
lib/pcg/test/src/pcg/machine_view.cc:28-300 (get_machine_space_coordinate):
per machine dimension (INTER_NODE = node index, INTRA_NODE = device index) the
task dimensions projected onto it form a mixed radix, first dimension
fastest, each digit weighted by its stride times the (degree x stride) of the
earlier dimensions on that projection; a coordinate that lands outside the
machine gives None."""
import json

import pytest

from flexflow_train_amd import _ffcore as C

INTRA, INTER = "INTRA_NODE", "INTER_NODE"


def _view(start, dims):
    return json.dumps({"start": list(start), "dimensions": [{"stride": s, "projection": p} for s, p in dims]})


def _coord(ts, view, coord, nodes, gpus):
    return C.get_machine_space_coordinate(ts, view, coord, C.MachineSpecification.mi355x(nodes, gpus))


# 1D: task space (3,), stride 2 on the device dimension from (0, 1), 1 node x 6 devices
ONE_D = ([3], _view((0, 1), [(2, INTRA)]), 1, 6)


@pytest.mark.parametrize("coord,want", [((0,), (0, 1)), ((1,), (0, 3)), ((2,), (0, 5)), ((4,), None)])
def test_1d(coord, want):
    ts, v, n, g = ONE_D
    assert _coord(ts, v, list(coord), n, g) == want


# 2D on different machine dimensions: (2, 2), node stride 1, device stride 2,
# start (1, 2), 3 nodes x 5 devices
TWO_D_DIFF = ([2, 2], _view((1, 2), [(1, INTER), (2, INTRA)]), 3, 5)


@pytest.mark.parametrize("coord,want", [((0, 0), (1, 2)), ((0, 1), (1, 4)), ((1, 0), (2, 2)), ((1, 1), (2, 4))])
def test_2d_different_dimensions(coord, want):
    ts, v, n, g = TWO_D_DIFF
    assert _coord(ts, v, list(coord), n, g) == want


# 2D on the same machine dimension: strides 1 and 2 on devices, start (1, 0),
# 2 nodes x 6 devices -> | (0,0) | (1,0) | . | . | (0,1) | (1,1) |
TWO_D_SAME = ([2, 2], _view((1, 0), [(1, INTRA), (2, INTRA)]), 2, 6)


@pytest.mark.parametrize("coord,want", [((0, 0), (1, 0)), ((0, 1), (1, 4)), ((1, 0), (1, 1)), ((1, 1), (1, 5))])
def test_2d_same_dimension(coord, want):
    ts, v, n, g = TWO_D_SAME
    assert _coord(ts, v, list(coord), n, g) == want


# 3D: node stride 1, device strides 2 and 1, start (0, 1), 2 nodes x 8 devices
THREE_D = ([2, 2, 2], _view((0, 1), [(1, INTER), (2, INTRA), (1, INTRA)]), 2, 8)


@pytest.mark.parametrize("coord,want", [((0, 1, 0), (0, 3)), ((1, 0, 1), (1, 5)), ((1, 1, 1), (1, 7))])
def test_3d(coord, want):
    ts, v, n, g = THREE_D
    assert _coord(ts, v, list(coord), n, g) == want


def test_device_ids_follow_coordinates():
    """get_device_ids lists node * gpus_per_node + device per task coordinate
    in row-major task order, and refuses a view that leaves the machine."""
    ts, v, n, g = THREE_D
    spec = C.MachineSpecification.mi355x(n, g)
    ids = C.get_device_ids(ts, v, spec)
    coords = [(a, b, c) for a in range(2) for b in range(2) for c in range(2)]
    assert ids == [(lambda m: m[0] * g + m[1])(_coord(ts, v, list(c), n, g)) for c in coords]
    with pytest.raises(Exception):
        C.get_device_ids([3], _view((0, 1), [(2, INTRA)]), C.MachineSpecification.mi355x(1, 4))


def test_allowed_views_all_fit():
    """Every allowed view of a 2-D task space fits the machine and is injective
    (allowed_machine_views.cc)."""
    spec = C.MachineSpecification.mi355x(2, 4)
    views = C.get_allowed_machine_views([2, 2], spec)
    assert views
    for v in views:
        ids = C.get_device_ids([2, 2], v, spec)
        assert len(set(ids)) == 4 and all(0 <= i < 8 for i in ids)


# ---- start-invariant views (start_invariant_machine_view.cc:9-229)
def test_start_invariant_conversions():
    mv = _view((1, 2), [(2, INTER), (3, INTRA)])
    simv = C.start_invariant_from_machine_view(mv)
    assert json.loads(simv) == {"dimensions": [{"stride": 2, "projection": INTER},
                                               {"stride": 3, "projection": INTRA}]}
    back = C.machine_view_from_start_invariant(simv, 1, 2)
    assert json.loads(back) == json.loads(mv)
    assert C.start_invariant_from_machine_view(back) == simv


@pytest.mark.parametrize("coord,want", [((0,), (0, 0)), ((1,), (0, 2)), ((2,), (0, 4))])
def test_start_invariant_offset_1d(coord, want):
    simv = json.dumps({"dimensions": [{"stride": 2, "projection": INTRA}]})
    assert C.get_machine_space_offset([3], simv, list(coord), C.MachineSpecification.mi355x(1, 6)) == want


@pytest.mark.parametrize("coord,want", [((0, 0), (0, 0)), ((0, 1), (0, 2)), ((1, 0), (1, 0)), ((1, 1), (1, 2))])
def test_start_invariant_offset_2d(coord, want):
    simv = json.dumps({"dimensions": [{"stride": 1, "projection": INTER}, {"stride": 2, "projection": INTRA}]})
    assert C.get_machine_space_offset([2, 2], simv, list(coord), C.MachineSpecification.mi355x(2, 4)) == want


# ---- get_allowed_machine_views (lib/compiler/test/src/allowed_machine_views.cc)
def _norm(v):
    j = json.loads(v)
    return tuple(j["start"]), tuple((d["stride"], d["projection"]) for d in j["dimensions"])


def test_allowed_views_one_degree():
    got = {_norm(v) for v in C.get_allowed_machine_views([3], C.MachineSpecification.mi355x(1, 5))}
    assert got == {((0, 0), ((1, INTRA),)), ((0, 1), ((1, INTRA),)), ((0, 2), ((1, INTRA),)),
                   ((0, 0), ((2, INTRA),))}


def test_allowed_views_two_degrees():
    got = {_norm(v) for v in C.get_allowed_machine_views([2, 3], C.MachineSpecification.mi355x(3, 3))}
    assert got == {((0, 0), ((1, INTER), (1, INTRA))), ((1, 0), ((1, INTER), (1, INTRA))),
                   ((0, 0), ((2, INTER), (1, INTRA))),
                   ((0, 0), ((1, INTRA), (1, INTER))), ((0, 1), ((1, INTRA), (1, INTER))),
                   ((0, 0), ((2, INTRA), (1, INTER)))}
