"""FFConfig: runtime configuration + the reference's command-line flag set.

Parity: lib/local-execution/include/local-execution/config.h:51-107 (FFConfig
fields) and bin/arg_parser/arg_parser.cc:5-153 (flags), python
FFConfig (python/flexflow/core/flexflow_cffi.py:526-566).  Legion-only flags
(-ll:*, -lg:*) are accepted and ignored; -ll:gpu maps to the number of GPUs
of the node (one process per GPU here: the world comes from torchrun's env).
"""
from __future__ import annotations

import argparse
import dataclasses
import os
import sys
import time
from typing import List, Optional


@dataclasses.dataclass
class FFConfig:
    epochs: int = 1
    batch_size: int = 64
    num_nodes: int = 1
    cpus_per_node: int = 1
    workers_per_node: int = 0          # GPUs per node (0 = from WORLD_SIZE / LOCAL_WORLD_SIZE)
    learning_rate: float = 0.01
    weight_decay: float = 0.0001
    print_freq: int = 10
    dataset_path: str = ""
    profiling: bool = False
    perform_fusion: bool = True
    search_budget: int = -1
    search_time_limit: float = 45.0    # seconds for the whole strategy search (MCMC + Unity + mapping)
    search_alpha: float = 1.2
    # a searched strategy replaces data parallelism only when its predicted
    # speedup reaches this (smaller predicted gains are within the cost model's error)
    search_min_speedup: float = 1.02
    search_overlap_backward_update: bool = True
    only_data_parallel: bool = False
    enable_parameter_parallel: bool = False
    enable_attribute_parallel: bool = False
    enable_inplace_optimizations: bool = False
    allow_tensor_op_math_conversion: bool = True
    import_strategy_file: str = ""
    export_strategy_file: str = ""
    export_strategy_task_graph_file: str = ""
    include_costs_dot_graph: bool = False
    export_strategy_computation_graph_file: str = ""
    # Unity rule set added to the built-in parallelization / fusion rules:
    # "" = the bundled TASO corpus (flexflow_train_amd/data/taso_rules.json,
    # docs/TASO_RULES.md), "none" = no rule set, else a legacy corpus JSON
    # (reference substitutions/*.json) or a substitution-set JSON
    substitution_json_path: str = ""
    machine_model_version: int = 0
    machine_model_file: str = ""
    simulator_segment_size: int = 16777216
    simulator_max_num_segments: int = 1
    simulator_work_space_size: int = 2 << 30
    search_num_nodes: int = -1
    search_num_workers: int = -1
    base_optimize_threshold: int = 10
    enable_control_replication: bool = True
    python_data_loader_type: int = 2
    enable_propagation: bool = False
    search_algorithm: str = "unity"    # unity | mcmc | data_parallel
    compute_dtype: str = "bfloat16"    # bfloat16 on GPU; CPU runs float unless asked
    seed: int = 0
    shard_optimizer: bool = False      # ZeRO-style sharded optimizer state (reduce-scatter + all-gather)
    bucket_mb: int = 64                # gradient all-reduce bucket size
    # micro-batches per optimizer step: fit() accumulates this many batches
    # (GPipe order, Executor.train_step_pipelined) before one update, and the
    # strategy search prices pipeline-parallel stage splits at that count
    micro_batches: int = 1
    enable_hipgraph: bool = True       # fit(): capture the training iteration as a hipGraph (1 GPU)
    device_arena: bool = False         # 1 GPU: the step allocates from a plan-sized device arena (runtime/arena.py)
    parameter_sync: str = "nccl"       # "nccl" (all-reduce) | "ps" (reference ParamSync::PS)
    cpu_only: bool = False             # run on the host even when a GPU is visible
    local_execution: bool = False      # train on the native C++ CPU executor (lib/local-execution parity)
    native_data_loader: bool = True    # fit() on arrays: C++ prefetcher + pinned async H2D (runtime/dataloader.py)
    shuffle_data: bool = False         # native loader: reshuffle the samples every epoch
    softmax_identity_backward: bool = False   # reference-parity softmax backward (a copy; docs/PARITY.md)
    # fault tolerance (the reference has neither): fit()
    # writes an atomic sharded checkpoint every `checkpoint_every` iterations
    # under `checkpoint_dir` (keeping the newest `keep_checkpoints`) and, when
    # started again (e.g. by torchrun --max-restarts after a failed rank),
    # resumes from the newest complete one at the iteration it recorded
    checkpoint_dir: str = ""
    checkpoint_every: int = 0
    keep_checkpoints: int = 2
    _start_time: float = dataclasses.field(default_factory=time.time)
    _models: list = dataclasses.field(default_factory=list, repr=False, compare=False)

    def __post_init__(self):
        pass

    # -- reference accessors -------------------------------------------------
    def parse_args(self, argv: Optional[List[str]] = None):
        argv = sys.argv[1:] if argv is None else argv
        p = build_arg_parser()
        ns, _unknown = p.parse_known_args(argv)
        for k, v in vars(ns).items():
            if v is not None and hasattr(self, k):
                setattr(self, k, v)
        return self

    def get_batch_size(self):
        return self.batch_size

    def get_workers_per_node(self):
        if self.workers_per_node:
            return self.workers_per_node
        return int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))

    def get_num_nodes(self):
        return self.num_nodes

    def get_epochs(self):
        return self.epochs

    def get_current_time(self):
        return (time.time() - self._start_time) * 1e6   # microseconds, like Legion's timer

    def begin_trace(self, trace_id: int):
        """Reference: Legion trace memoisation around one iteration.  Here the
        FFModels built on this config capture the traced iteration as a
        hipGraph (second occurrence) and replay it afterwards."""
        for m in self._models:
            m._trace_begin(trace_id)

    def end_trace(self, trace_id: int):
        for m in self._models:
            m._trace_end(trace_id)


def build_arg_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(add_help=False, allow_abbrev=False)
    a = p.add_argument
    a("-e", "--epochs", dest="epochs", type=int)
    a("-b", "--batch-size", dest="batch_size", type=int)
    a("--lr", "--learning-rate", dest="learning_rate", type=float)
    a("--wd", "--weight-decay", dest="weight_decay", type=float)
    a("-p", "--print-freq", dest="print_freq", type=int)
    a("-d", "--dataset", dest="dataset_path", type=str)
    a("--budget", "--search-budget", dest="search_budget", type=int)
    a("--search-time-limit", dest="search_time_limit", type=float)
    a("--alpha", "--search-alpha", dest="search_alpha", type=float)
    a("--search-min-speedup", dest="search_min_speedup", type=float)
    a("--simulator-workspace-size", dest="simulator_work_space_size", type=int)
    a("--import", "--import-strategy", dest="import_strategy_file", type=str)
    a("--export", "--export-strategy", dest="export_strategy_file", type=str)
    a("--only-data-parallel", dest="only_data_parallel", action="store_const", const=True)
    a("--enable-parameter-parallel", dest="enable_parameter_parallel", action="store_const", const=True)
    a("--enable-attribute-parallel", dest="enable_attribute_parallel", action="store_const", const=True)
    a("-ll:gpu", dest="workers_per_node", type=int)
    a("--nodes", dest="num_nodes", type=int)
    a("-ll:cpu", dest="cpus_per_node", type=int)
    a("--profiling", dest="profiling", action="store_const", const=True)
    a("--allow-tensor-op-math-conversion", dest="allow_tensor_op_math_conversion", action="store_const",
      const=True)
    a("--fusion", dest="perform_fusion", action="store_const", const=True)
    a("--overlap", dest="search_overlap_backward_update", action="store_const", const=True)
    a("--taskgraph", dest="export_strategy_task_graph_file", type=str)
    a("--include-costs-dot-graph", dest="include_costs_dot_graph", action="store_const", const=True)
    a("--compgraph", dest="export_strategy_computation_graph_file", type=str)
    a("--machine-model-version", dest="machine_model_version", type=int)
    a("--machine-model-file", dest="machine_model_file", type=str)
    a("--simulator-segment-size", dest="simulator_segment_size", type=int)
    a("--simulator-max-num-segments", dest="simulator_max_num_segments", type=int)
    a("--enable-propagation", dest="enable_propagation", action="store_const", const=True)
    a("--enable-inplace-optimizations", dest="enable_inplace_optimizations", action="store_const", const=True)
    a("--search-num-nodes", dest="search_num_nodes", type=int)
    a("--search-num-workers", dest="search_num_workers", type=int)
    a("--base-optimize-threshold", dest="base_optimize_threshold", type=int)
    a("--disable-control-replication", dest="enable_control_replication", action="store_const", const=False)
    a("--python-data-loader-type", dest="python_data_loader_type", type=int)
    a("--substitution-json", dest="substitution_json_path", type=str)
    a("--search-algorithm", dest="search_algorithm", type=str)
    a("--compute-dtype", dest="compute_dtype", type=str)
    a("--shard-optimizer", "--zero", dest="shard_optimizer", action="store_const", const=True)
    a("--bucket-mb", dest="bucket_mb", type=int)
    a("--micro-batches", dest="micro_batches", type=int)
    a("--disable-hipgraph", dest="enable_hipgraph", action="store_const", const=False)
    a("--device-arena", dest="device_arena", action="store_const", const=True)
    a("--python-data-loader", dest="native_data_loader", action="store_const", const=False)
    a("--local-execution", dest="local_execution", action="store_const", const=True)
    a("--cpu", dest="cpu_only", action="store_const", const=True)
    a("--param-sync", dest="parameter_sync", choices=["nccl", "ps"])
    a("--shuffle", dest="shuffle_data", action="store_const", const=True)
    a("--softmax-identity-backward", dest="softmax_identity_backward", action="store_const", const=True)
    a("--seed", dest="seed", type=int)
    a("--checkpoint-dir", dest="checkpoint_dir", type=str)
    a("--checkpoint-every", dest="checkpoint_every", type=int)
    a("--keep-checkpoints", dest="keep_checkpoints", type=int)
    # Legion / Realm flags: accepted, ignored
    for f in ("-ll:fsize", "-ll:zsize", "-ll:util", "-ll:bgwork", "-ll:csize", "-lg:prof", "-lg:prof_logfile"):
        a(f, dest="_ignored_" + f.strip("-").replace(":", "_"), type=str)
    return p


class NetConfig:
    """Dataset location of the CNN examples (reference flexflow_cffi.py:2400
    NetConfig: the ``--dataset`` / ``-d`` flag)."""

    def __init__(self, argv: Optional[List[str]] = None):
        ns, _ = build_arg_parser().parse_known_args(sys.argv[1:] if argv is None else argv)
        self.dataset_path = ns.dataset_path or ""


def flexflow_python_binding() -> str:
    """The reference selects cffi / pybind11 bindings; this framework's
    native core is bound with pybind11."""
    return "pybind11"


def flexflow_python_interpreter() -> str:
    return "native"

