"""Native replay of segmented distributed steps (csrc/runtime/replay.cpp,
``_ffreplay``).  On the CPU: the collective path of the C++ walker against
torch.distributed over gloo at world size 2 (all-reduce, broadcast, reduce,
all-to-all through the c10d ProcessGroup the executor's DistContext hands
over), async slots and waits, and the recorder's descriptor plumbing.  The
graph launches and RCCL run in tests/test_rccl_gpu.py (world 1, nccl)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

R = pytest.importorskip("flexflow_train_amd._ffreplay")


def test_kinds_match_recorder():
    from flexflow_train_amd.runtime import graphs as G
    assert G.NATIVE_KINDS == {"all_reduce": R.ALL_REDUCE, "reduce_scatter": R.REDUCE_SCATTER,
                              "all_gather": R.ALL_GATHER, "reduce": R.REDUCE, "broadcast": R.BROADCAST,
                              "all_to_all": R.ALL_TO_ALL}
    rp = R.Replayer()
    rp.add_wait(0)          # waiting on a slot never issued is a no-op
    rp.replay()
    assert len(rp) == 1 and rp.n_graphs() == 0


def test_recorder_needs_descriptors():
    from flexflow_train_amd.runtime.graphs import SegmentRecorder
    rec = SegmentRecorder.__new__(SegmentRecorder)   # no capture pool on the CPU
    rec.items, rec.cur, rec.n_async, rec._native = [], None, 0, None
    rec.begin = lambda: None
    rec.collective(lambda: None, False)              # no descriptor -> Python walk
    assert rec.build_native() is False and not rec.native


_CHILD = r'''
import os, sys, json
sys.path.insert(0, ROOT)
import torch, torch.distributed as dist
from flexflow_train_amd import _ffreplay as R
from flexflow_train_amd.parallel.comm import DistContext
dist.init_process_group("gloo")
ctx = DistContext.from_env()
r, w = ctx.rank, ctx.world
pg = ctx._pg(None)
a = torch.arange(8, dtype=torch.float32) + 10 * r
b = torch.full((8,), float(r + 1))
c = torch.full((8,), float(r + 5))
send = torch.arange(4, dtype=torch.float32) + 100 * r
recv = torch.empty(4)
rp = R.Replayer()
rp.add_collective(R.ALL_REDUCE, pg, a, a, 0, 0)          # async slot 0
rp.add_wait(0)
rp.add_collective(R.BROADCAST, pg, b, b, ctx._group_rank(None, 1), -1)
rp.add_collective(R.REDUCE, pg, c, c, 0, 1)             # async slot 1, waited at the end
rp.add_collective(R.ALL_TO_ALL, pg, send, recv, 0, -1, [2, 2], [2, 2])
rp.replay()
print(json.dumps({"a": a.tolist(), "b": b.tolist(), "c": c.tolist(), "recv": recv.tolist()}))
dist.destroy_process_group()
'''


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_native_collectives_gloo_world2():
    import json
    port = _port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        code = f"ROOT = {ROOT!r}\n" + _CHILD
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e[-3000:]
        outs.append(json.loads(o.strip().splitlines()[-1]))
    base = torch.arange(8, dtype=torch.float32)
    for rank, o in enumerate(outs):
        assert o["a"] == (2 * base + 10).tolist()                # sum over ranks
        assert o["b"] == [2.0] * 8                              # rank 1's values
        if rank == 0:
            assert o["c"] == [5.0 + 6.0] * 8                    # reduced into rank 0
        # all-to-all: rank r gets elements [2r, 2r+1] of every rank's send buffer
        want = [100.0 * s + 2 * rank + j for s in range(2) for j in range(2)]
        assert o["recv"] == want
