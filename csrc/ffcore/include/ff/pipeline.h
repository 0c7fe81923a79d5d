// Pipeline parallelism as a search candidate: the model's operators cut into
// S contiguous stages (balanced by their costed forward + backward time),
// each stage data-parallel over its own block of world / S devices, trained
// on m micro-batches per optimizer step in a GPipe / 1F1B schedule.
//
// Parity: the reference has no pipeline search (PIPELINE exists
// only as an OperatorType); Unity's inter-operator placement via machine
// views is the closest.  Here the stage assignment, the micro-batch count and
// the bubble are priced next to the Unity / MCMC strategies by the same cost
// model, at equal work (m micro-batches per step for every strategy):
//
//   pipeline step = (m + S - 1) * max_s (fwd + bwd of stage s + its boundary
//                   sends, per micro-batch)            <- fill / drain bubble
//                 + max_s gradient all-reduce of stage s over its block
//                 + max_s optimizer update of stage s
//   other strategy = m * backward_end + (iteration - backward_end)
//                   (the simulator's one-batch timeline, the forward/backward
//                   part repeated per micro-batch, one sync + update)
//
// 1F1B and GPipe share the step time; they differ in the activations a stage
// keeps live: m micro-batches (GPipe) vs min(m, S - s) (1F1B).
#pragma once
#include <map>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/machine.h"
#include "ff/memory_plan.h"
#include "ff/simulator.h"

namespace ff {

struct PipelinePlan {
  int stages = 1;
  int micro_batches = 1;
  int stage_degree = 1;                 // data-parallel degree inside a stage
  std::vector<double> stage_time;       // per micro-batch: fwd + bwd + boundary sends (s)
  std::vector<double> stage_sync;       // gradient all-reduce per stage (s)
  std::vector<double> stage_update;     // optimizer update per stage (s)
  std::vector<double> stage_activation_bytes;  // saved activations per micro-batch
  double step_time = 0;                 // one optimizer step (m micro-batches)
  double bubble_fraction = 0;           // (S - 1) / (m + S - 1)
  ParallelComputationGraph pcg;         // data-parallel at stage_degree
  std::map<int, int> stage_of;          // PCG node -> stage
  std::map<int, Placement> views;       // PCG node -> its stage's device block
  Json to_json(bool with_views = false) const;
};

// memory plan config of a pipeline plan: stage s keeps min(m, S - s) micro-
// batches of activations live under 1F1B, m under GPipe
MemoryPlanConfig pipeline_memory_config(const PipelinePlan& p, bool one_f_one_b = true);

// one optimizer step of m micro-batches under a non-pipelined strategy
double micro_batched_step_time(const SimResult& one_batch, int micro_batches);

// S stages on `world` devices (world % S == 0), m micro-batches
PipelinePlan price_pipeline(const ComputationGraph& cg, const CostModel& cm, int world, int stages,
                            int micro_batches, const SimConfig& sim);
// every S >= 2 dividing world (and at most the number of operators)
std::vector<PipelinePlan> pipeline_candidates(const ComputationGraph& cg, const CostModel& cm, int world,
                                              int micro_batches, const SimConfig& sim);

}  // namespace ff
