"""The task-graph simulator (csrc/ffcore/src/simulator.cc) on schedules
small enough to compute by hand: region-intersection transfers between
placements (a cross-device move, a 2-way repartition edge, replicas),
routed transfers over the network topology, parameter-server
synchronization (reduce -> leader update -> broadcast) and the bucketed
all-reduce pass.  Reference: lib/runtime/src/simulator.cc:843-899 (region
intersections), :957-1019 (PS tasks), :1087-1215 (NCCL pass),
:1245-1870 (routed LogicalTaskgraph transfers)."""
import json

import pytest

from flexflow_train_amd import _ffcore as C
from flexflow_train_amd.core import ActiMode, DataType, FFConfig, FFModel
from flexflow_train_amd.search import native

XGMI = 64e9
LAT = 8e-6


def _shape(sizes, degrees, s=1, c=1):
    return C.ParallelTensorShape(list(sizes), list(degrees), s, c, C.DataType.FLOAT)


def _chain(batch=64, hidden=256):
    m = FFModel(FFConfig())
    x = m.create_tensor([batch, hidden], DataType.DT_FLOAT, name="x")
    t = m.dense(x, hidden, ActiMode.AC_MODE_RELU, name="a")
    t = m.dense(t, hidden, name="b")
    m.softmax(t, name="sm")
    return m


def _tasks(res):
    return res["tasks"]


def test_region_transfers_cross_move_repartition_and_replicas():
    t = _shape([8, 4], [2, 1])                       # two pieces of 4 x 4 floats = 64 B each
    assert C.region_transfers(t, [0, 1], [0, 1]) == []
    # a 2-way repartition edge whose pieces swap devices: each device receives the other's piece
    assert sorted(C.region_transfers(t, [0, 1], [1, 0])) == [(0, 1, 64.0), (1, 0, 64.0)]
    # placement widened with implicit replicas: devices 2 and 3 read from the holders
    assert sorted(C.region_transfers(t, [0, 1], [0, 2, 1, 3])) == [(0, 2, 64.0), (1, 3, 64.0)]
    # a whole (degree-1) tensor moved from device 0 to device 1
    u = _shape([8, 4], [1, 1])
    assert C.region_transfers(u, [0], [1]) == [(0, 1, 128.0)]


def test_cross_device_move_schedule():
    """Producer on device 0, consumer on device 1: one transfer of the whole
    activation between them (bytes / xGMI link + latency); the consumer's
    forward starts when it lands; the gradient flows back the same way."""
    m = _chain()
    pcg = C.data_parallel_pcg(m.cg, 1)
    names = {pcg.layer_name(n): n for n in pcg.topo_order()}
    views = {n: [0] for n in pcg.topo_order()}
    for nm in ("b", "sm"):
        views[names[nm]] = [1]
    for n in pcg.topo_order():
        if pcg.is_weight_path(n) and pcg.layer_name(n).startswith("b."):
            views[n] = [1]
    cm = native.cost_model(use_profiles=False)
    r = native.simulate(pcg, cm, 2, views, dot=True)
    ts = _tasks(r)
    fwd = {t["name"]: t for t in ts if t["name"].endswith(":fwd")}
    xs = [t for t in ts if t["type"] == 5]
    assert r["num_xfers"] == 2 and len(xs) == 2           # activation forward, gradient backward
    x_f = next(t for t in xs if t["name"] == "b:in")
    nbytes = 64 * 256 * 4
    assert (x_f["src"], x_f["dst"], x_f["bytes"]) == (0, 1, nbytes)
    assert x_f["end"] - x_f["start"] == pytest.approx(nbytes / XGMI + LAT)
    assert x_f["start"] == pytest.approx(fwd["a:fwd"]["end"])
    assert fwd["b:fwd"]["start"] == pytest.approx(x_f["end"])
    x_b = next(t for t in xs if t["name"] == "a:grad")
    assert (x_b["src"], x_b["dst"]) == (1, 0)
    bwd = {t["name"]: t for t in ts if t["name"].endswith(":bwd")}
    assert x_b["start"] == pytest.approx(bwd["b:bwd"]["end"])
    assert bwd["a:bwd"]["start"] >= x_b["end"] - 1e-12
    assert r["xfer_bytes"] == pytest.approx(2 * nbytes)


def test_routed_transfer_occupies_route_links():
    """With a network model a transfer takes its route: inside an MI355X node
    one xGMI link; across nodes GPU -> NIC switch -> GPU (two links)."""
    m = _chain()
    pcg = C.data_parallel_pcg(m.cg, 1)
    names = {pcg.layer_name(n): n for n in pcg.topo_order()}
    cm = native.cost_model(use_profiles=False)
    net = C.NetworkModel(C.NetworkTopology.mi355x_cluster(2))
    for dst, hops in ((5, 1), (9, 2)):
        views = {n: [0] for n in pcg.topo_order()}
        for n in pcg.topo_order():
            if pcg.layer_name(n).split(".")[0] in ("b", "sm"):
                views[n] = [dst]
        r = native.simulate(pcg, cm, 16, views, dot=True, network=net)
        x_f = next(t for t in _tasks(r) if t["type"] == 5 and t["name"] == "b:in")
        assert len(x_f["links"]) == hops, x_f
        assert x_f["end"] - x_f["start"] == pytest.approx(net.p2p_time(0, dst, x_f["bytes"]))


def test_parameter_server_tasks():
    """ParamSync::PS: each replicated weight's gradients are reduced into the
    group leader (comm lane), the leader updates, the weights go back; no
    all-reduce and no per-device update task."""
    m = _chain()
    pcg = C.data_parallel_pcg(m.cg, 2)
    cm = native.cost_model(use_profiles=False)
    ps = native.simulate(pcg, cm, 2, dot=True, parameter_server=True)
    nccl = native.simulate(pcg, cm, 2, dot=True)
    kinds = [t["type"] for t in _tasks(ps)]
    assert 4 not in kinds                                  # no ALLREDUCE
    reduces = [t for t in _tasks(ps) if t["type"] == 6]
    bcasts = [t for t in _tasks(ps) if t["type"] == 7]
    updates = [t for t in _tasks(ps) if t["type"] == 3]
    assert len(reduces) == len(bcasts) == len(updates) == 4   # a / b kernels and biases
    for rd in reduces:
        up = next(u for u in updates if rd["name"].replace("ps_reduce", "ps_update") == u["name"])
        bc = next(b for b in bcasts if rd["name"].replace("ps_reduce", "ps_bcast") == b["name"])
        assert up["devices"] == [0]                           # the group leader
        assert up["start"] >= rd["end"] - 1e-12 and bc["start"] >= up["end"] - 1e-12
    # hand-computed: a's kernel (256 x 256 fp32 grads, bf16 for the GEMM weight) over 2 copies
    rk = next(t for t in reduces if t["name"] == "a:ps_reduce0")
    bk = next(t for t in bcasts if t["name"] == "a:ps_bcast0")
    gather = 256 * 256 * 2 / XGMI + LAT      # one peer's bf16 kernel gradient into the leader
    bcast = 256 * 256 * 4 / XGMI + LAT       # the fp32 kernel back to it
    assert rk["end"] - rk["start"] == pytest.approx(gather)
    assert bk["end"] - bk["start"] == pytest.approx(bcast)
    assert ps["iteration_time"] >= max(b["end"] for b in bcasts) - 1e-12
    assert any(t["type"] == 4 for t in _tasks(nccl))
    assert ps["sync_time"] > 0 and bcast > 0


def test_nccl_buckets_serialize_on_comm_lane():
    m = _chain(batch=256, hidden=2048)
    pcg = C.data_parallel_pcg(m.cg, 4)
    cm = native.cost_model(use_profiles=False)
    r = native.simulate(pcg, cm, 4, dot=True, bucket_bytes=1.0)   # one bucket per weight
    ars = sorted((t for t in _tasks(r) if t["type"] == 4), key=lambda t: t["start"])
    assert len(ars) >= 4
    for a, b in zip(ars, ars[1:]):
        assert b["start"] >= a["end"] - 1e-12                    # one RCCL stream per device
    ups = [t for t in _tasks(r) if t["type"] == 3]
    assert len(ups) == 4 and all(u["start"] >= ars[-1]["end"] - 1e-12 for u in ups)


def test_pipeline_stages_overlap_in_simulation():
    """Two stages on different devices with a transfer between them: the
    iteration costs at least both stages plus the hop (no overlap within one
    micro-batch), and the dot export names the transfer."""
    m = _chain()
    pcg = C.data_parallel_pcg(m.cg, 1)
    views = {}
    for n in pcg.topo_order():
        views[n] = [1] if pcg.layer_name(n).split(".")[0] in ("b", "sm") else [0]
    cm = native.cost_model(use_profiles=False)
    r = native.simulate(pcg, cm, 2, views, dot=True)
    assert "XFER 0->1" in r["dot"]
    one = native.simulate(pcg, cm, 1)
    assert r["iteration_time"] > one["iteration_time"]


def test_measured_memory_drives_peak():
    """Profile entries with allocator measurements (resident_mb / peak_mb,
    search/profiler.py) replace the analytic activation bytes; the largest
    transient workspace of a device is added once (it is not resident)."""
    from flexflow_train_amd.search.profiler import collect_signatures
    m = _chain()
    pcg = C.data_parallel_pcg(m.cg, 1)
    cm = native.cost_model(use_profiles=False)
    base = native.simulate(pcg, cm, 1)["peak_memory"]
    sigs = collect_signatures([pcg])
    table = {}
    for i, sig in enumerate(sigs):
        table[sig] = {"fwd_ms": 0.01, "bwd_ms": 0.02, "resident_mb": 100.0 * (i + 1), "peak_mb": 100.0 * (i + 1) + 50.0 * i}
    cm2 = native.cost_model(use_profiles=False)
    cm2.load_profiles(json.dumps(table))
    got = native.simulate(pcg, cm2, 1)["peak_memory"]
    n = len(sigs)
    resident = sum(100e6 * (i + 1) for i in range(n))
    workspace = 50e6 * (n - 1)
    # weights (bf16 copy + fp32 master + Adam m, v + grad = 16 B / param) stay analytic
    weights = 2 * (256 * 256 + 256) * 16.0
    assert got == pytest.approx(weights + resident + workspace)
    assert base > weights      # analytic activations before
    assert json.loads(cm2.profiles_json())[next(iter(sigs))]["peak_mb"] == pytest.approx(100.0)


def test_executor_fusions_priced():
    """The executor runs residual add + LayerNorm as one kernel and the final
    softmax inside the softmax + cross-entropy loss: with executor_fusions the
    simulator prices the add at zero (one extra input read in the norm) and
    the final softmax as one read + one write of the logits, no backward."""
    m = FFModel(FFConfig())
    x = m.create_tensor([4096, 1024], DataType.DT_FLOAT, name="x")
    h = m.dense(x, 1024, name="proj")
    t = m.layer_norm(m.add(x, h, name="res"), [1], True, 1e-5, name="ln")
    m.softmax(m.dense(t, 4096, name="head"), name="sm")
    pcg = C.data_parallel_pcg(m.cg, 1)
    cm = native.cost_model(world=1, use_profiles=False)
    fused = native.simulate(pcg, cm, 1, dot=True)
    plain = native.simulate(pcg, cm, 1, dot=True, executor_fusions=False)
    assert fused["iteration_time"] < plain["iteration_time"]

    def run(res, name):
        return sum(t["end"] - t["start"] for t in res["tasks"] if t["name"].split(":")[0] == name and t["type"] in (0, 1))
    names = {pcg.layer_name(n): n for n in pcg.topo_order()}
    assert "res" in names and "sm" in names
    assert run(fused, "res") == 0.0 and run(plain, "res") > 0.0
    assert run(fused, "ln") > run(plain, "ln")               # the extra input read
    logits = 4096 * 4096 * 4                                  # fp32 piece of the head output
    hbm = cm.spec().hbm_bandwidth
    assert run(fused, "sm") == pytest.approx(2 * logits / hbm + cm.spec().kernel_launch_overhead, rel=1e-6)
    assert run(plain, "sm") > run(fused, "sm")
