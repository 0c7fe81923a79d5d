"""Step-by-step probe of the device arena under torch's MemPool (prints each
stage before it runs, so a crash names its stage)."""
import sys

import torch


def say(*a):
    print(*a, flush=True)


say("1 cuda init")
torch.cuda.init()
x = torch.empty(16, device="cuda")
say("2 arena reserve")
from flexflow_train_amd.runtime import arena as A  # noqa: E402
import ctypes  # noqa: E402
lib = ctypes.CDLL(A._LIB)
lib.ff_arena_reserve.argtypes = [ctypes.c_int, ctypes.c_size_t]
say("   rc", lib.ff_arena_reserve(0, 256 << 20))
say("3 pluggable allocator")
alloc = torch.cuda.memory.CUDAPluggableAllocator(A._LIB, "ff_arena_alloc", "ff_arena_free")
say("4 mempool")
pool = torch.cuda.MemPool(alloc.allocator())
say("   pool id", pool.id)
say("5 allocate in pool")
with torch.cuda.use_mem_pool(pool):
    y = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
say("   sum", float(y.sum()))
say("6 graph capture into pool")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    z = y * 2
with torch.cuda.graph(g, pool=pool.id):
    z = y * 2 + 1
g.replay()
torch.cuda.synchronize()
say("   z", float(z.sum()))
say("7 done")
sys.exit(0)
