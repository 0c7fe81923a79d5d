// The training-backing interface behind the legacy C API
// (csrc/ffi/flexflow_runtime_c.cc): one process, one device, a
// ComputationGraph trained step by step with tensors reachable as host slots.
// Two implementations:
//  * LocalTrainingBacking (ff/local_exec.h) -- the native CPU executor;
//  * the GPU backing (csrc/ffdev/device_exec.cpp, make_device_backing) --
//    device buffers, hand-written HIP kernels (exact-fp32 MFMA GEMMs,
//    softmax + cross-entropy, MSE) and host slots kept as mirrors that are
//    copied in / out on demand (the reference's inline-mapped regions).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "ff/computation_graph.h"

namespace ff {

struct HostTensor {
  std::vector<int64_t> dims;
  std::vector<float> v;
  int64_t numel() const { return static_cast<int64_t>(v.size()); }
  void resize(const std::vector<int64_t>& d);
};

struct LocalOptimizer {
  std::string kind = "sgd";  // sgd | adam
  double lr = 0.01, momentum = 0.0, weight_decay = 0.0;
  bool nesterov = false;
  double beta1 = 0.9, beta2 = 0.999, epsilon = 1e-8;
};

struct LocalMetrics {
  double loss_sum = 0.0;
  int64_t correct = 0, samples = 0;
};

class TrainingBacking {
 public:
  virtual ~TrainingBacking() = default;
  // the slot of any graph tensor (or its gradient) as a host buffer; nullptr
  // if none is kept.  A device backing copies the current contents out and
  // treats the slot as written by the caller (copied back before the next
  // device step).
  virtual HostTensor* slot(const ValueRef& v, bool grad = false) = 0;
  virtual ValueRef output() const = 0;
  virtual LocalOptimizer& optimizer() = 0;
  virtual void forward_layer(int node) = 0;
  virtual void forward() = 0;
  // loss + metrics on the output, then the full backward pass
  virtual void backward(const std::vector<float>& labels) = 0;
  virtual void update() = 0;
  virtual const LocalMetrics& metrics() const = 0;
  virtual void reset_metrics() = 0;
  // "cpu" or "gpu:<ordinal>"
  virtual std::string device() const = 0;
};

// The GPU backing when a GPU is visible and every operator of `cg` has a
// device implementation (else nullptr: the caller keeps the CPU backing).
// `why` (optional) receives the reason when nullptr is returned.  Defined in
// csrc/ffdev/device_exec.cpp, which libflexflow_runtime_c links.
std::unique_ptr<TrainingBacking> make_device_backing(const ComputationGraph& cg, LocalOptimizer opt,
                                                     const std::string& loss, uint64_t seed, std::string* why);

}  // namespace ff
