"""Joint substitution + parallelization search entry point (filled in by the
native search; until the cost model is wired this returns data parallel)."""
from .. import _ffcore as C


def search(cg, ffconfig, world):
    pcg = C.data_parallel_pcg(cg, world)
    return pcg, {}, {"source": "data_parallel_fallback"}
