"""The reference's protobuf strategy files (examples/cpp/DLRM/strategies/
*.pb, FFProtoBuf::Strategy): byte-exact decode/encode of the shipped files,
lowering onto a DLRM (one table per GPU + data-parallel MLPs), and a 2-rank
gloo run of an imported .pb strategy that must match the single-process
run parameter for parameter."""
import os

import pytest

import dist_models as M
from dist_util import assert_params_close, run_distributed, run_single
from flexflow_train_amd.search import legacy_strategy as L

REF = "/root/reference/examples/cpp/DLRM/strategies"


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
@pytest.mark.parametrize("fname", ["dlrm_strategy_8embs_8gpus.pb", "dlrm_strategy_16embs_8gpus.pb",
                                   "dlrm_strategy_16embs_16gpus.pb"])
def test_reference_pb_roundtrip(fname):
    data = open(os.path.join(REF, fname), "rb").read()
    ops = L.decode(data)
    assert L.encode(ops) == data
    embs = [o for o in ops if o["name"].startswith("embedding")]
    assert embs and all(o["dims"] == [1, 1] and len(o["device_ids"]) == 1 for o in embs)


def _dlrm8(m):
    from flexflow_train_amd.models.recsys import DLRMConfig, build_dlrm
    build_dlrm(m, DLRMConfig(batch_size=64, embedding_size=[100] * 8, sparse_feature_size=16,
                             mlp_bot=[8, 16, 16], mlp_top=[16, 16, 2]))


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not mounted")
def test_lower_reference_dlrm_strategy():
    from flexflow_train_amd import _ffcore as C
    from flexflow_train_amd.core import FFConfig, FFModel

    m = FFModel(FFConfig())
    _dlrm8(m)
    ops = L.decode(open(os.path.join(REF, "dlrm_strategy_8embs_8gpus.pb"), "rb").read())
    pcg, views, rep = L.to_pcg(m.cg, ops, 8)
    assert rep["matched_layers"] >= 8 + 1
    tables = [n for n in pcg.topo_order() if pcg.layer_op(n).op_type == "EMBEDDING"]
    assert sorted(views[n] for n in tables) == [(i,) for i in range(8)]
    for n in tables:   # each table whole on its device (degree 1)
        assert pcg.shape(C.ValueRef(n, 0)).total_parallel_degree() == 1
    with pytest.raises(ValueError):
        L.to_pcg(m.cg, ops, 4)   # device ids beyond the world


def test_exported_pb_reimports(tmp_path):
    from flexflow_train_amd.core import FFConfig, FFModel
    from flexflow_train_amd.search.strategy import export_strategy

    m = FFModel(FFConfig())
    M.dlrm_small(m)
    ops = [{"name": f"embedding{i}", "dims": [1, 1], "device_ids": [i % 2]} for i in range(4)]
    ops += [{"name": "linear", "dims": [1, 2], "device_ids": [0, 1]}]
    pcg, views, _ = L.to_pcg(m.cg, ops, 2)
    path = str(tmp_path / "s.pb")
    export_strategy(path, pcg, views)
    back = L.decode(open(path, "rb").read())
    by = {o["name"]: o for o in back}
    assert [by[f"emb{i}"]["device_ids"] for i in range(4)] == [[0], [1], [0], [1]]
    assert by["top0"]["dims"] == [1, 2]
    pcg2, views2, _ = L.to_pcg(m.cg, back, 2)
    assert views2 == views


def test_imported_pb_strategy_trains_like_single_process(tmp_path):
    """Tables alternate between the 2 ranks (the reference generator's
    ``i % gpus``), everything else data parallel."""
    ops = [{"name": f"embedding{i}", "device_type": "GPU", "dims": [1, 1], "device_ids": [i % 2]}
           for i in range(4)]
    for nm in ("linear", "concat", "mse_loss"):
        ops.append({"name": nm, "device_type": "GPU", "dims": [1, 2], "device_ids": [0, 1]})
    path = str(tmp_path / "dlrm_strategy_4embs_2gpus.pb")
    with open(path, "wb") as f:
        f.write(L.encode(ops))
    ref = run_single(M.dlrm_small, steps=2)
    out = run_distributed(M.dlrm_small, 2, path, steps=2)
    assert_params_close(out["params"], ref["params"])
    assert out["stats"]["all_to_all"] + out["stats"].get("p2p", 0) + out["stats"].get("send_recv", 0) > 0   # tables -> DP concat exchange
