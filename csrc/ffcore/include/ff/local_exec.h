// Native single-device CPU executor of a ComputationGraph: the MI355X
// framework's counterpart of the reference's lib/local-execution.
//
// Parity:
//  * LocalTrainingBacking (local_training_backing.cc:50-163): topo-order
//    forward, reverse backward, per-layer elapsed ms — plus the update step the
//    reference leaves unimplemented;
//  * task registry / signatures (task_registry.cc, task_signature_impl.cc,
//    op_task_signature.cc): an OpType -> {forward, backward} table over plain
//    slot views instead of Legion-era privilege bindings;
//  * slots backing (local_slots_backing.cc:20-172): one host buffer per
//    tensor and per gradient (created only where gradients are needed);
//  * LocalCostEstimator (local_cost_estimator.cc:29-105): `measure_op` runs an
//    operator alone on synthetic inputs of the given shapes and times it;
//  * loss / metrics functions (loss_function_kernels.cu, metrics_functions.cu)
//    and fused SGD / Adam (optimizer_kernel.cu) on the host.
// BASELINE config 1 ("MNIST MLP via lib/local-execution on CPU") runs here.
// fp32 throughout; integer index tensors are carried as floats.
#pragma once
#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/training_backing.h"

namespace ff {

class LocalTrainingBacking : public TrainingBacking {
 public:
  // loss: "sparse_categorical_crossentropy" | "categorical_crossentropy" |
  // "mean_squared_error" | "identity"
  LocalTrainingBacking(const ComputationGraph& cg, LocalOptimizer opt, std::string loss, uint64_t seed = 0,
                       bool input_grads = false);

  std::vector<std::string> input_names() const;
  std::vector<std::string> weight_names() const;
  std::vector<int64_t> shape_of(const std::string& name) const;  // input / weight / layer output
  void set_input(const std::string& name, const std::vector<float>& data);
  void set_weight(const std::string& name, const std::vector<float>& data);
  std::vector<float> get_weight(const std::string& name) const;
  std::vector<float> get_output() const;  // the graph's (last layer's) output
  ValueRef output() const override { return output_; }
  // the slot of any graph tensor (or its gradient); nullptr if none is kept
  HostTensor* slot(const ValueRef& v, bool grad = false) override;
  LocalOptimizer& optimizer() override { return opt_; }
  // runs one operator layer's forward on the current slot contents
  void forward_layer(int node) override;

  void forward() override;
  // loss + metrics on the output, then the full backward pass
  void backward(const std::vector<float>& labels) override;
  void update() override;
  void train_step(const std::vector<float>& labels) {
    forward();
    backward(labels);
    update();
  }
  const LocalMetrics& metrics() const override { return metrics_; }
  void reset_metrics() override { metrics_ = LocalMetrics{}; }
  std::string device() const override { return "cpu"; }
  // operator layers in topo order / whether a tensor carries a gradient
  const std::vector<int>& order() const { return order_; }
  bool needs_grad(const ValueRef& v) const {
    auto it = needs_grad_.find(v);
    return it != needs_grad_.end() && it->second;
  }
  const std::string& loss() const { return loss_; }
  bool fused_softmax_ce() const { return fused_softmax_ce_; }
  // per layer name: accumulated forward / backward milliseconds
  std::map<std::string, std::pair<double, double>> layer_times_ms() const;

  struct OpCtx {
    const OpAttrs* op;
    std::vector<HostTensor*> in, w, out;
    std::vector<HostTensor*> d_in, d_w, d_out;  // nullptr where no gradient is kept
    std::vector<HostTensor>* saved;             // per-layer scratch kept from fwd to bwd
    bool training = true;
    uint64_t seed = 0;
  };
  using Fn = std::function<void(OpCtx&)>;
  struct OpImpl {
    Fn fwd, bwd;
  };
  static const std::map<OpType, OpImpl>& registry();

 private:
  void init_weight(int node, HostTensor& t, const std::string& init_json, uint64_t seed);
  const ComputationGraph& cg_;
  LocalOptimizer opt_;
  std::string loss_;
  uint64_t seed_;
  std::vector<int> order_;                         // operator layers in topo order
  std::map<ValueRef, HostTensor> val_, grad_;      // slots: tensors and gradients
  std::map<ValueRef, bool> needs_grad_;
  std::map<int, std::vector<HostTensor>> saved_;
  std::map<std::string, int> input_of_, weight_of_;
  std::map<int, HostTensor> m1_, m2_;              // optimizer state per weight node
  int64_t step_ = 0;
  ValueRef output_;
  bool fused_softmax_ce_ = false;
  LocalMetrics metrics_;
  std::map<int, std::pair<double, double>> times_;
};

// LocalCostEstimator: forward + backward milliseconds of one operator on
// synthetic inputs of `input_shapes` (median of `iters` runs after a warm-up).
double measure_op_cost_ms(const OpAttrs& op, const std::vector<TensorShape>& input_shapes, int iters = 3);

}  // namespace ff
