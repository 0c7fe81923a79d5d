// Static memory plan of one training step from tensor liveness.
//
// The reference sizes Legion regions per tensor and leaves reuse to the
// runtime's instance GC; its simulator adds every op's tensors
// (simulator.cc:1216-1242).  Here each device gets an explicit plan over
// the step's schedule -- forward in topological order, backward in reverse:
//   * an activation lives from its producer's forward until its producer's
//     backward (consumers save their inputs for the backward, and the
//     producer may need its output), or only until its last forward reader
//     when nothing is trained;
//   * an activation gradient lives from the backward of its last consumer
//     (the first to produce a contribution) to its producer's backward;
//   * weights, weight gradients and optimizer state stay resident
//     (`weight_bytes_per_param` each, 16 = bf16 copy + fp32 master + Adam m, v
//     + bf16 gradient, as the cost model counts);
// and the blocks are packed into one arena by first-fit-decreasing offsets
// over the interval graph (blocks whose lifetimes overlap never share
// bytes).  `peak_live_bytes` is the lower bound (max over time of the live
// sum), `arena_bytes` what the packing achieves, `naive_bytes` the sum the
// per-op accounting would give.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/json.h"
#include "ff/machine.h"

namespace ff {

struct MemBlock {
  int node = -1;
  int output = 0;
  int kind = 0;          // 0 activation, 1 activation gradient, 2 weights + state
  double bytes = 0;
  int start = 0, end = 0;  // schedule steps [start, end], inclusive
  double offset = 0;       // in the device arena
};

struct MemoryPlan {
  int device = 0;
  int steps = 0;
  double weight_bytes = 0, peak_live_bytes = 0, arena_bytes = 0, naive_bytes = 0;
  std::vector<MemBlock> blocks;
  Json to_json(bool with_blocks = false) const;
};

struct MemoryPlanConfig {
  bool training = true;
  double weight_bytes_per_param = 16.0;
  double align = 256.0;   // bytes
  // activations of node n held live `live_copies[n]` times (default 1): a
  // pipeline stage keeps the saved activations of several micro-batches
  // (1F1B: min(m, S - s) on stage s, GPipe: m)
  std::map<int, double> live_copies;
  // bytes per activation / activation-gradient element as the executor
  // stores them (2: bf16 compute); 0 = the PCG tensor's own dtype
  double act_elem_bytes = 0.0;
  // the executor's fusions and saved tensors (runtime/executor.py, the op
  // implementations), measured by tools/mem_audit.py
  // (profiles/r6/g04_mem_audit_*.jsonl):
  //  * BATCHNORM (no ReLU) -> EW_ADD -> RELU runs as one kernel: the BN and
  //    add outputs (and their gradients) never exist;
  //  * the final SOFTMAX is fused with the loss: no softmax output, and the
  //    logits' gradient overwrites the logits (no separate block);
  //  * LINEAR with an activation keeps its pre-activation too (x2);
  //  * MULTIHEAD_ATTENTION keeps the q / k / v projections and the
  //    attention output (flash attention: no score matrix) beside its output;
  //  * an output that neither its producer's nor any consumer's backward
  //    reads is freed after its last forward reader (the executor drops it
  //    from its environment); otherwise it lives until its last reader's
  //    backward
  bool executor_fusions = false;
};

// one plan per device 0 .. world-1
std::vector<MemoryPlan> plan_memory(const ParallelComputationGraph& pcg, const std::map<int, Placement>& views,
                                    int world, const MemoryPlanConfig& cfg = {});

}  // namespace ff
