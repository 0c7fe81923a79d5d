// Legacy FFModel runtime C API (see flexflow_runtime_c.h) over the native
// ComputationGraph + LocalTrainingBacking.
//
// Parity: python/flexflow_c.cc of the reference (the cffi surface of its
// Python package): the same entry points, argument order and enum values.
// Differences by design: tensors live in host slots of the backing instead
// of Legion regions, so inline map / raw pointers hand out the slot itself
// (zero copy for fp32; int32 views are converted on unmap), and the model
// runs single-process (the multi-GPU runtime is the Python executor).
#include "flexflow_runtime_c.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "ff/computation_graph.h"
#include "ff/local_exec.h"

namespace {

thread_local std::string g_err;
std::vector<std::string> g_args;  // begin_flexflow_task / config_parse_args

void set_error(const std::string& m) {
  g_err = m;
  std::fprintf(stderr, "flexflow_runtime: %s\n", m.c_str());
}

std::string nm(const char* s) { return s ? std::string(s) : std::string(); }

struct RtConfig {
  int batch_size = 64, epochs = 1, workers_per_node = 1, num_nodes = 1, loader_type = 2;
  double lr = 0.01, weight_decay = 0.0001;
  bool only_data_parallel = false, control_replication = true;
  std::string dataset;
  void parse(const std::vector<std::string>& a) {
    auto next = [&](size_t& i) { return i + 1 < a.size() ? a[++i] : std::string(); };
    for (size_t i = 0; i < a.size(); ++i) {
      const std::string& f = a[i];
      if (f == "-b" || f == "--batch-size") batch_size = std::atoi(next(i).c_str());
      else if (f == "-e" || f == "--epochs") epochs = std::atoi(next(i).c_str());
      else if (f == "--lr" || f == "--learning-rate") lr = std::atof(next(i).c_str());
      else if (f == "--wd" || f == "--weight-decay") weight_decay = std::atof(next(i).c_str());
      else if (f == "--nodes") num_nodes = std::atoi(next(i).c_str());
      else if (f == "-ll:gpu") workers_per_node = std::atoi(next(i).c_str());
      else if (f == "--only-data-parallel") only_data_parallel = true;
      else if (f == "--disable-control-replication") control_replication = false;
      else if (f == "--python-data-loader-type") loader_type = std::atoi(next(i).c_str());
      else if (f == "-d" || f == "--dataset") dataset = next(i);
    }
  }
};

struct RtModel;

struct RtTensor {
  RtModel* m = nullptr;
  ff::ValueRef v{-1, 0};
  std::vector<int64_t> dims;         // outermost first
  ff::DataType dtype = ff::DataType::FLOAT;
  std::vector<float> staging;        // data before compile (and the label tensor)
  std::vector<int32_t> i32;          // int32 view handed out by get_raw_ptr_int32
  std::vector<int> legion_dims;      // innermost first (get_dims)
  bool mapped = false;
  int64_t numel() const {
    int64_t n = 1;
    for (auto d : dims) n *= d;
    return n;
  }
};

struct RtOp {
  RtModel* m = nullptr;
  int node = -1;
};

struct RtOptimizer {
  ff::LocalOptimizer o;
  RtModel* m = nullptr;
};

struct RtInit {
  std::string json;
};

struct RtMetrics {
  int64_t correct = 0, all = 0;
  double loss = 0;
};

struct RtModel {
  RtConfig cfg;
  ff::ComputationGraph cg;
  std::unique_ptr<ff::TrainingBacking> be;
  std::string device = "cpu", device_note;
  ff::LocalOptimizer opt;
  std::string loss = "sparse_categorical_crossentropy";
  bool sparse_labels = true;
  std::map<ff::ValueRef, std::unique_ptr<RtTensor>> tensors;
  std::map<int, std::unique_ptr<RtOp>> ops;
  std::vector<int> layers;  // operator layers in creation order
  std::unique_ptr<RtTensor> label;
  int traces = 0;

  RtTensor* wrap(ff::ValueRef v) {
    auto& t = tensors[v];
    if (!t) {
      t = std::make_unique<RtTensor>();
      t->m = this;
      t->v = v;
      const auto& s = cg.shape(v);
      t->dims = s.dims;
      t->dtype = s.dtype;
      for (auto it = s.dims.rbegin(); it != s.dims.rend(); ++it) t->legion_dims.push_back(static_cast<int>(*it));
    }
    return t.get();
  }
  RtOp* op(int node) {
    auto& o = ops[node];
    if (!o) {
      o = std::make_unique<RtOp>();
      o->m = this;
      o->node = node;
    }
    return o.get();
  }
  void added(const std::vector<ff::ValueRef>& outs) {
    if (be) throw std::runtime_error("layers cannot be added after compile()");
    if (!outs.empty()) layers.push_back(outs[0].node);
  }
  // the float storage of a tensor (or its gradient); nullptr if none exists
  float* data(RtTensor* t, bool grad) {
    if (t == label.get()) return grad ? nullptr : t->staging.data();
    if (be) {
      auto* s = be->slot(t->v, grad);
      if (s) return s->v.data();
      if (grad) return nullptr;
    }
    if (grad) return nullptr;
    if (t->staging.empty()) t->staging.assign(t->numel(), 0.f);
    return t->staging.data();
  }
};

template <typename T>
T* impl(void* p, const char* what) {
  if (!p) throw std::invalid_argument(std::string("null ") + what + " handle");
  return static_cast<T*>(p);
}
RtModel* M(flexflow_model_t h) { return impl<RtModel>(h.impl, "model"); }
RtTensor* T(flexflow_tensor_t h) { return impl<RtTensor>(h.impl, "tensor"); }
RtConfig* CFG(flexflow_config_t h) { return impl<RtConfig>(h.impl, "config"); }
flexflow_tensor_t wrapT(RtTensor* t) { return flexflow_tensor_t{t}; }
flexflow_tensor_t nullT() { return flexflow_tensor_t{nullptr}; }

std::string init_json(flexflow_initializer_t i) {
  return i.impl ? static_cast<RtInit*>(i.impl)->json : std::string();
}

ff::Activation act(int a) {
  switch (a) {
    case AC_MODE_RELU: return ff::Activation::RELU;
    case AC_MODE_SIGMOID: return ff::Activation::SIGMOID;
    case AC_MODE_TANH: return ff::Activation::TANH;
    case AC_MODE_GELU: return ff::Activation::GELU;
    default: return ff::Activation::NONE;
  }
}

ff::DataType dtype_of(int d) {
  switch (d) {
    case DT_BOOLEAN: return ff::DataType::BOOL;
    case DT_INT32: return ff::DataType::INT32;
    case DT_INT64: return ff::DataType::INT64;
    case DT_HALF: return ff::DataType::HALF;
    case DT_DOUBLE: return ff::DataType::DOUBLE;
    case DT_NONE: return ff::DataType::NONE;
    default: return ff::DataType::FLOAT;
  }
}
int dtype_enum(ff::DataType d) {
  switch (d) {
    case ff::DataType::BOOL: return DT_BOOLEAN;
    case ff::DataType::INT32: return DT_INT32;
    case ff::DataType::INT64: return DT_INT64;
    case ff::DataType::HALF: return DT_HALF;
    case ff::DataType::DOUBLE: return DT_DOUBLE;
    case ff::DataType::NONE: return DT_NONE;
    default: return DT_FLOAT;
  }
}

// runs f; on an exception records it and returns `fallback`
template <typename R, typename F>
R guard(R fallback, F&& f) {
  try {
    return f();
  } catch (const std::exception& e) {
    set_error(e.what());
    return fallback;
  }
}
template <typename F>
void guard_void(F&& f) {
  try {
    f();
  } catch (const std::exception& e) {
    set_error(e.what());
  }
}

std::vector<int64_t> ints(const int* p, int n) {
  std::vector<int64_t> r;
  for (int i = 0; i < n; ++i) r.push_back(p[i]);
  return r;
}

flexflow_tensor_t unary(flexflow_model_t h, ff::OpType t, flexflow_tensor_t x, const char* name,
                        std::optional<double> s = {}) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.unary(t, T(x)->v, nm(name), s);
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t binary(flexflow_model_t h, ff::OpType t, flexflow_tensor_t a, flexflow_tensor_t b,
                         const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.binary(t, T(a)->v, T(b)->v, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}

bool copy_in(RtTensor* t, const float* src, int64_t n) {
  if (n != t->numel()) throw std::invalid_argument("tensor size mismatch");
  std::memcpy(t->m->data(t, false), src, sizeof(float) * static_cast<size_t>(n));
  return true;
}
int64_t count(int num_dim, const int* dims) {
  int64_t n = 1;
  for (int i = 0; i < num_dim; ++i) n *= dims[i];
  return n;
}

std::vector<int> int_list(const std::vector<int>& v) {
  std::vector<int> r{static_cast<int>(v.size())};
  r.insert(r.end(), v.begin(), v.end());
  return r;
}
std::vector<int> dash_list(const std::string& s) {
  std::vector<int> r;
  std::stringstream ss(s);
  std::string w;
  while (std::getline(ss, w, '-'))
    if (!w.empty()) r.push_back(std::atoi(w.c_str()));
  return r;
}

struct RtNetConfig {
  std::string dataset;
  RtNetConfig() {
    for (size_t i = 0; i + 1 < g_args.size(); ++i)
      if (g_args[i] == "--dataset") dataset = g_args[i + 1];
  }
};

struct RtDLRMConfig {
  int sparse_feature_size = 2, sigmoid_bot = -1, sigmoid_top = -1, embedding_bag_size = 1;
  float loss_threshold = 0.f;
  std::string interaction = "cat", dataset;
  std::vector<int> embedding_size{4}, mlp_bot{4, 2}, mlp_top{8, 2};
  std::vector<int> out_emb, out_bot, out_top;  // count-prefixed copies handed out
  RtDLRMConfig() {
    for (size_t i = 0; i + 1 < g_args.size(); ++i) {
      const std::string& f = g_args[i];
      const std::string& v = g_args[i + 1];
      if (f == "--arch-sparse-feature-size") sparse_feature_size = std::atoi(v.c_str());
      else if (f == "--arch-embedding-size") embedding_size = dash_list(v);
      else if (f == "--embedding-bag-size") embedding_bag_size = std::atoi(v.c_str());
      else if (f == "--arch-mlp-bot") mlp_bot = dash_list(v);
      else if (f == "--arch-mlp-top") mlp_top = dash_list(v);
      else if (f == "--loss-threshold") loss_threshold = static_cast<float>(std::atof(v.c_str()));
      else if (f == "--sigmoid-top") sigmoid_top = std::atoi(v.c_str());
      else if (f == "--sigmoid-bot") sigmoid_bot = std::atoi(v.c_str());
      else if (f == "--arch-interaction-op") interaction = v;
      else if (f == "--dataset") dataset = v;
    }
  }
};

struct RtLoader {
  RtModel* m = nullptr;
  RtTensor* batch = nullptr;
  std::vector<float> full;  // num_samples x sample
  int64_t num_samples = 0, sample = 0, next = 0;
  // integer samples (embedding ids) are staged in the runtime's fp32 tensor
  // storage: exact only up to 2^24, so larger ids are refused instead of
  // silently rounded onto a neighbouring row
  static float exact_id(int64_t v) {
    if (v > (int64_t{1} << 24) || v < -(int64_t{1} << 24))
      throw std::invalid_argument("dataloader: integer sample " + std::to_string(v) +
                                  " exceeds 2^24 and cannot be stored exactly");
    return static_cast<float>(v);
  }
  void load(const void* src, int dt, int64_t n) {
    full.resize(static_cast<size_t>(n));
    if (dt == DT_INT32) {
      auto p = static_cast<const int32_t*>(src);
      for (int64_t i = 0; i < n; ++i) full[i] = exact_id(p[i]);
    } else if (dt == DT_INT64) {
      auto p = static_cast<const int64_t*>(src);
      for (int64_t i = 0; i < n; ++i) full[i] = exact_id(p[i]);
    } else {
      std::memcpy(full.data(), src, sizeof(float) * static_cast<size_t>(n));
    }
  }
  void next_batch() {
    const int64_t bs = batch->dims.empty() ? 1 : batch->dims[0];
    float* dst = m->data(batch, false);
    for (int64_t r = 0; r < bs; ++r) {
      const int64_t idx = (next + r) % std::max<int64_t>(1, num_samples);
      std::memcpy(dst + r * sample, full.data() + idx * sample, sizeof(float) * static_cast<size_t>(sample));
    }
    next += bs;
  }
};

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" {

const char* flexflow_runtime_last_error(void) { return g_err.c_str(); }

const char* flexflow_model_get_device(flexflow_model_t h) {
  static thread_local std::string out;
  out.clear();
  guard_void([&] {
    auto* m = M(h);
    out = m->be ? m->device : "uncompiled";
    if (m->be && m->device == "cpu" && !m->device_note.empty()) out += " (" + m->device_note + ")";
  });
  return out.c_str();
}

// ---- FFConfig ------------------------------------------------------------
flexflow_config_t flexflow_config_create(void) {
  auto* c = new RtConfig();
  c->parse(g_args);
  return flexflow_config_t{c};
}
void flexflow_config_destroy(flexflow_config_t h) { delete static_cast<RtConfig*>(h.impl); }
void flexflow_config_parse_args(flexflow_config_t h, char** argv, int argc) {
  guard_void([&] {
    std::vector<std::string> a;
    for (int i = 0; i < argc; ++i) a.emplace_back(argv[i] ? argv[i] : "");
    CFG(h)->parse(a);
    g_args = a;
  });
}
void flexflow_config_parse_args_default(flexflow_config_t h) {
  guard_void([&] { CFG(h)->parse(g_args); });
}
int flexflow_config_get_batch_size(flexflow_config_t h) { return guard(-1, [&] { return CFG(h)->batch_size; }); }
int flexflow_config_get_workers_per_node(flexflow_config_t h) {
  return guard(-1, [&] { return CFG(h)->workers_per_node; });
}
int flexflow_config_get_num_nodes(flexflow_config_t h) { return guard(-1, [&] { return CFG(h)->num_nodes; }); }
int flexflow_config_get_epochs(flexflow_config_t h) { return guard(-1, [&] { return CFG(h)->epochs; }); }
bool flexflow_config_get_enable_control_replication(flexflow_config_t h) {
  return guard(false, [&] { return CFG(h)->control_replication; });
}
int flexflow_config_get_python_data_loader_type(flexflow_config_t h) {
  return guard(-1, [&] { return CFG(h)->loader_type; });
}

// ---- FFModel -------------------------------------------------------------
flexflow_model_t flexflow_model_create(flexflow_config_t config) {
  return guard(flexflow_model_t{nullptr}, [&] {
    auto* m = new RtModel();
    m->cfg = *CFG(config);
    m->opt.lr = m->cfg.lr;
    m->opt.weight_decay = m->cfg.weight_decay;
    return flexflow_model_t{m};
  });
}
void flexflow_model_destroy(flexflow_model_t h) { delete static_cast<RtModel*>(h.impl); }
void flexflow_model_reset_metrics(flexflow_model_t h) {
  guard_void([&] {
    if (M(h)->be) M(h)->be->reset_metrics();
  });
}
void flexflow_model_init_layers(flexflow_model_t h) {
  guard_void([&] {
    if (!M(h)->be) throw std::runtime_error("init_layers before compile()");
  });
}
void flexflow_model_prefetch(flexflow_model_t) {}
void flexflow_model_forward(flexflow_model_t h, int) {
  guard_void([&] {
    auto* m = M(h);
    if (!m->be) throw std::runtime_error("forward before compile()");
    m->be->forward();
  });
}
void flexflow_model_backward(flexflow_model_t h, int) {
  guard_void([&] {
    auto* m = M(h);
    if (!m->be) throw std::runtime_error("backward before compile()");
    m->be->backward(m->label->staging);
  });
}
void flexflow_model_compute_metrics(flexflow_model_t h) {
  // loss and metrics are accumulated by backward() (LocalTrainingBacking)
  guard_void([&] { (void)M(h); });
}
void flexflow_model_update(flexflow_model_t h) {
  guard_void([&] {
    auto* m = M(h);
    if (!m->be) throw std::runtime_error("update before compile()");
    m->be->optimizer() = m->opt;
    m->be->update();
  });
}
void flexflow_model_compile(flexflow_model_t h, enum LossType loss_type, int*, int, enum CompMode) {
  guard_void([&] {
    auto* m = M(h);
    switch (loss_type) {
      case LOSS_CATEGORICAL_CROSSENTROPY: m->loss = "categorical_crossentropy"; break;
      case LOSS_SPARSE_CATEGORICAL_CROSSENTROPY: m->loss = "sparse_categorical_crossentropy"; break;
      case LOSS_MEAN_SQUARED_ERROR_AVG_REDUCE:
      case LOSS_MEAN_SQUARED_ERROR_SUM_REDUCE: m->loss = "mean_squared_error"; break;
      default: m->loss = "identity";
    }
    m->sparse_labels = loss_type == LOSS_SPARSE_CATEGORICAL_CROSSENTROPY;
    // the GPU backing when a GPU is visible and every operator has a device
    // implementation (FF_C_API_DEVICE=cpu keeps the host), else the CPU one
    m->be = ff::make_device_backing(m->cg, m->opt, m->loss, 0, &m->device_note);
    if (!m->be) m->be = std::make_unique<ff::LocalTrainingBacking>(m->cg, m->opt, m->loss, 0);
    m->device = m->be->device();
    // data written before compile moves into the backing's slots
    for (auto& kv : m->tensors) {
      RtTensor* t = kv.second.get();
      if (t->staging.empty()) continue;
      if (auto* s = m->be->slot(t->v, false)) {
        if (static_cast<int64_t>(t->staging.size()) == s->numel()) s->v = t->staging;
      }
      t->staging.clear();
      t->staging.shrink_to_fit();
    }
    auto lab = std::make_unique<RtTensor>();
    lab->m = m;
    lab->dims = m->cg.shape(m->be->output()).dims;
    if (m->sparse_labels && !lab->dims.empty()) lab->dims.back() = 1;
    lab->dtype = m->sparse_labels ? ff::DataType::INT32 : ff::DataType::FLOAT;
    for (auto it = lab->dims.rbegin(); it != lab->dims.rend(); ++it) lab->legion_dims.push_back(static_cast<int>(*it));
    lab->staging.assign(lab->numel(), 0.f);
    m->label = std::move(lab);
  });
}
flexflow_tensor_t flexflow_model_get_label_tensor(flexflow_model_t h) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    if (!m->label) throw std::runtime_error("label tensor before compile()");
    return wrapT(m->label.get());
  });
}
void flexflow_model_zero_gradients(flexflow_model_t h) {
  guard_void([&] {
    auto* m = M(h);
    if (!m->be) return;
    for (auto& kv : m->tensors)
      if (auto* g = m->be->slot(kv.first, true)) std::fill(g->v.begin(), g->v.end(), 0.f);
  });
}

flexflow_tensor_t flexflow_model_add_exp(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, ff::OpType::EXP, x, name);
}
flexflow_tensor_t flexflow_model_add_sin(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, ff::OpType::SIN, x, name);
}
flexflow_tensor_t flexflow_model_add_cos(flexflow_model_t h, const flexflow_tensor_t x, const char* name) {
  return unary(h, ff::OpType::COS, x, name);
}
flexflow_tensor_t flexflow_model_add_add(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool, const char* name) {
  return binary(h, ff::OpType::EW_ADD, x, y, name);
}
flexflow_tensor_t flexflow_model_add_subtract(flexflow_model_t h, const flexflow_tensor_t x,
                                              const flexflow_tensor_t y, bool, const char* name) {
  return binary(h, ff::OpType::EW_SUB, x, y, name);
}
flexflow_tensor_t flexflow_model_add_multiply(flexflow_model_t h, const flexflow_tensor_t x,
                                              const flexflow_tensor_t y, bool, const char* name) {
  return binary(h, ff::OpType::EW_MUL, x, y, name);
}
flexflow_tensor_t flexflow_model_add_divide(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                            bool, const char* name) {
  return binary(h, ff::OpType::EW_DIV, x, y, name);
}
flexflow_tensor_t flexflow_model_add_max(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool, const char* name) {
  return binary(h, ff::OpType::EW_MAX, x, y, name);
}
flexflow_tensor_t flexflow_model_add_min(flexflow_model_t h, const flexflow_tensor_t x, const flexflow_tensor_t y,
                                         bool, const char* name) {
  return binary(h, ff::OpType::EW_MIN, x, y, name);
}
flexflow_tensor_t flexflow_model_add_reduce_sum(flexflow_model_t h, const flexflow_tensor_t input, int* axes, int n,
                                                bool keepdims, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.reduce(ff::OpType::REDUCE_SUM, T(input)->v, ints(axes, n), keepdims, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_rsqrt(flexflow_model_t h, const flexflow_tensor_t input, const char* name) {
  return unary(h, ff::OpType::RSQRT, input, name);
}
flexflow_tensor_t flexflow_model_add_pow(flexflow_model_t h, const flexflow_tensor_t input, const float exponent,
                                         const char* name) {
  return unary(h, ff::OpType::POW, input, name, static_cast<double>(exponent));
}
flexflow_tensor_t flexflow_model_add_mean(flexflow_model_t h, const flexflow_tensor_t input, int* dims, int n,
                                          bool keepdims, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.reduce(ff::OpType::MEAN, T(input)->v, ints(dims, n), keepdims, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_relu(flexflow_model_t h, const flexflow_tensor_t input, bool,
                                          const char* name) {
  return unary(h, ff::OpType::RELU, input, name);
}
flexflow_tensor_t flexflow_model_add_scalar_multiply(flexflow_model_t h, const flexflow_tensor_t input,
                                                     const float scalar, bool, const char* name) {
  return unary(h, ff::OpType::SCALAR_MULTIPLY, input, name, static_cast<double>(scalar));
}
flexflow_tensor_t flexflow_model_add_scalar_add(flexflow_model_t h, const flexflow_tensor_t input, const float scalar,
                                                bool, const char* name) {
  return unary(h, ff::OpType::SCALAR_ADD, input, name, static_cast<double>(scalar));
}
flexflow_tensor_t flexflow_model_add_scalar_sub(flexflow_model_t h, const flexflow_tensor_t input, const float scalar,
                                                bool, const char* name) {
  return unary(h, ff::OpType::SCALAR_SUB, input, name, static_cast<double>(scalar));
}
flexflow_tensor_t flexflow_model_add_scalar_truediv(flexflow_model_t h, const flexflow_tensor_t input,
                                                    const float scalar, bool, const char* name) {
  return unary(h, ff::OpType::SCALAR_TRUE_DIV, input, name, static_cast<double>(scalar));
}
flexflow_tensor_t flexflow_model_add_gelu(flexflow_model_t h, const flexflow_tensor_t input, const char* name) {
  return unary(h, ff::OpType::GELU, input, name);
}
flexflow_tensor_t flexflow_model_add_identity(flexflow_model_t h, const flexflow_tensor_t input, const char* name) {
  return unary(h, ff::OpType::IDENTITY, input, name);
}
flexflow_tensor_t flexflow_model_add_sigmoid(flexflow_model_t h, const flexflow_tensor_t input, const char* name) {
  return unary(h, ff::OpType::SIGMOID, input, name);
}
flexflow_tensor_t flexflow_model_add_tanh(flexflow_model_t h, const flexflow_tensor_t input, const char* name) {
  return unary(h, ff::OpType::TANH, input, name);
}
flexflow_tensor_t flexflow_model_add_elu(flexflow_model_t h, const flexflow_tensor_t input, bool, const char* name) {
  return unary(h, ff::OpType::ELU, input, name);
}
flexflow_tensor_t flexflow_model_add_dropout(flexflow_model_t h, const flexflow_tensor_t input, float rate,
                                             unsigned long long seed, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.dropout(T(input)->v, rate, static_cast<int64_t>(seed), nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}

flexflow_tensor_t flexflow_model_add_conv2d(flexflow_model_t h, const flexflow_tensor_t input, int out_channels,
                                            int kernel_h, int kernel_w, int stride_h, int stride_w, int padding_h,
                                            int padding_w, enum ActiMode activation, int groups, bool use_bias,
                                            flexflow_op_t shared_op, flexflow_initializer_t kernel_initializer,
                                            flexflow_initializer_t bias_initializer, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    ff::OpAttrs a(ff::OpType::CONV2D);
    a.set("out_channels", static_cast<int64_t>(out_channels)).set("kernel_h", kernel_h).set("kernel_w", kernel_w);
    a.set("stride_h", stride_h).set("stride_w", stride_w).set("padding_h", padding_h).set("padding_w", padding_w);
    a.set("groups", groups).set("activation", ff::to_string(act(activation))).set("use_bias", use_bias);
    std::vector<ff::ValueRef> outs;
    if (shared_op.impl)
      outs = m->cg.add_layer_with_weights(a, {T(input)->v},
                                          m->cg.layer_weights(static_cast<RtOp*>(shared_op.impl)->node), nm(name));
    else
      outs = m->cg.add_layer(a, {T(input)->v}, nm(name), {init_json(kernel_initializer), init_json(bias_initializer)});
    m->added(outs);
    return wrapT(m->wrap(outs[0]));
  });
}
flexflow_tensor_t flexflow_model_add_embedding(flexflow_model_t h, const flexflow_tensor_t input, int num_entires,
                                               int out_dim, enum AggrMode aggr, flexflow_op_t shared_op,
                                               flexflow_initializer_t kernel_initializer, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    const std::string ag = aggr == AGGR_MODE_SUM ? "sum" : aggr == AGGR_MODE_AVG ? "avg" : "none";
    ff::ValueRef v;
    if (shared_op.impl) {
      ff::OpAttrs a(ff::OpType::EMBEDDING);
      a.set("num_entries", static_cast<int64_t>(num_entires)).set("out_channels", static_cast<int64_t>(out_dim));
      a.set("aggr", ag).set("data_type", ff::to_string(ff::DataType::FLOAT));
      v = m->cg.add_layer_with_weights(a, {T(input)->v},
                                       m->cg.layer_weights(static_cast<RtOp*>(shared_op.impl)->node), nm(name))[0];
    } else {
      v = m->cg.embedding(T(input)->v, num_entires, out_dim, ag, ff::DataType::FLOAT, nm(name),
                          init_json(kernel_initializer));
    }
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_pool2d(flexflow_model_t h, flexflow_tensor_t input, int kernel_h, int kernel_w,
                                            int stride_h, int stride_w, int padding_h, int padding_w,
                                            enum PoolType type, enum ActiMode activation, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.pool2d(T(input)->v, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                          type == POOL_AVG ? "avg" : "max", act(activation), nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_batch_norm(flexflow_model_t h, const flexflow_tensor_t input, bool relu,
                                                const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.batch_norm(T(input)->v, relu, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_layer_norm(flexflow_model_t h, const flexflow_tensor_t input, int n, int* axes,
                                                bool elementwise_affine, float eps, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.layer_norm(T(input)->v, ints(axes, n), elementwise_affine, eps, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_batch_matmul(flexflow_model_t h, const flexflow_tensor_t a,
                                                  const flexflow_tensor_t b, int, int) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.batch_matmul(T(a)->v, T(b)->v, "");
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_dense(flexflow_model_t h, const flexflow_tensor_t input, int out_dim,
                                           enum ActiMode activation, bool use_bias, enum DataType,
                                           flexflow_op_t shared_op, flexflow_initializer_t kernel_initializer,
                                           flexflow_initializer_t bias_initializer, enum RegularizerMode kernel_reg_type,
                                           float kernel_reg_lambda, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    ff::ValueRef v;
    if (shared_op.impl) {
      ff::OpAttrs a(ff::OpType::LINEAR);
      a.set("out_channels", static_cast<int64_t>(out_dim)).set("use_bias", use_bias);
      a.set("activation", ff::to_string(act(activation)));
      v = m->cg.add_layer_with_weights(a, {T(input)->v},
                                       m->cg.layer_weights(static_cast<RtOp*>(shared_op.impl)->node), nm(name))[0];
    } else {
      v = m->cg.dense(T(input)->v, out_dim, act(activation), use_bias, nm(name), init_json(kernel_initializer),
                      init_json(bias_initializer));
    }
    if (kernel_reg_type == REG_MODE_L2 && kernel_reg_lambda > 0.f)
      m->opt.weight_decay = std::max(m->opt.weight_decay, static_cast<double>(kernel_reg_lambda));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_concat(flexflow_model_t h, int n, flexflow_tensor_t* input, int axis,
                                            const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    std::vector<ff::ValueRef> xs;
    for (int i = 0; i < n; ++i) xs.push_back(T(input[i])->v);
    auto v = m->cg.concat(xs, axis, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
void flexflow_model_add_split(flexflow_model_t h, flexflow_tensor_t input, int n, flexflow_tensor_t* outputs,
                              int* split, int axis, const char* name) {
  guard_void([&] {
    auto* m = M(h);
    auto vs = m->cg.split(T(input)->v, ints(split, n), axis, nm(name));
    m->added(vs);
    for (int i = 0; i < n; ++i) outputs[i] = wrapT(m->wrap(vs[i]));
  });
}
flexflow_tensor_t flexflow_model_add_flat(flexflow_model_t h, flexflow_tensor_t input, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.flat(T(input)->v, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_gather(flexflow_model_t h, const flexflow_tensor_t input,
                                            const flexflow_tensor_t index, int dim, const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.gather(T(input)->v, T(index)->v, dim, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_softmax(flexflow_model_t h, const flexflow_tensor_t input, int dim,
                                             const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.softmax(T(input)->v, dim, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_transpose(flexflow_model_t h, const flexflow_tensor_t input, int n, int* perm,
                                               const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.transpose(T(input)->v, ints(perm, n), nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_reshape(flexflow_model_t h, const flexflow_tensor_t input, int n, int* shape,
                                             const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.reshape(T(input)->v, ints(shape, n), nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_reverse(flexflow_model_t h, const flexflow_tensor_t input, int axis,
                                             const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    auto v = m->cg.reverse(T(input)->v, axis, nm(name));
    m->added({v});
    return wrapT(m->wrap(v));
  });
}
flexflow_tensor_t flexflow_model_add_multihead_attention(flexflow_model_t h, const flexflow_tensor_t query,
                                                         const flexflow_tensor_t key, const flexflow_tensor_t value,
                                                         int embed_dim, int num_heads, int kdim, int vdim,
                                                         float dropout, bool bias, bool add_bias_kv,
                                                         bool add_zero_attn, flexflow_initializer_t kernel_initializer,
                                                         const char* name) {
  return guard(nullT(), [&] {
    auto* m = M(h);
    if (add_bias_kv || add_zero_attn) throw std::invalid_argument("add_bias_kv / add_zero_attn are not supported");
    ff::OpAttrs a(ff::OpType::MULTIHEAD_ATTENTION);
    a.set("embed_dim", static_cast<int64_t>(embed_dim)).set("num_heads", static_cast<int64_t>(num_heads));
    a.set("kdim", static_cast<int64_t>(kdim)).set("vdim", static_cast<int64_t>(vdim));
    a.set("dropout", static_cast<double>(dropout)).set("bias", bias);
    auto outs = m->cg.add_layer(a, {T(query)->v, T(key)->v, T(value)->v}, nm(name), {init_json(kernel_initializer)});
    m->added(outs);
    return wrapT(m->wrap(outs[0]));
  });
}

void flexflow_model_set_sgd_optimizer(flexflow_model_t h, flexflow_sgd_optimizer_t optimizer) {
  guard_void([&] {
    M(h)->opt = impl<RtOptimizer>(optimizer.impl, "optimizer")->o;
    static_cast<RtOptimizer*>(optimizer.impl)->m = M(h);
  });
}
void flexflow_model_set_adam_optimizer(flexflow_model_t h, flexflow_adam_optimizer_t optimizer) {
  guard_void([&] {
    M(h)->opt = impl<RtOptimizer>(optimizer.impl, "optimizer")->o;
    static_cast<RtOptimizer*>(optimizer.impl)->m = M(h);
  });
}
void flexflow_model_print_layers(flexflow_model_t h, int id) {
  guard_void([&] {
    auto* m = M(h);
    for (size_t i = 0; i < m->layers.size(); ++i) {
      if (id >= 0 && static_cast<int>(i) != id) continue;
      const auto& node = m->cg.g.node(m->layers[i]);
      std::printf("layer %zu %s %s", i, node.label.name.c_str(), ff::to_string(node.label.op.type).c_str());
      for (auto const& o : node.outputs) {
        std::printf(" [");
        for (size_t d = 0; d < o.shape.dims.size(); ++d)
          std::printf("%s%lld", d ? ", " : "", static_cast<long long>(o.shape.dims[d]));
        std::printf("]");
      }
      std::printf("\n");
    }
  });
}
flexflow_op_t flexflow_model_get_layer_by_id(flexflow_model_t h, int layer_id) {
  return guard(flexflow_op_t{nullptr}, [&] {
    auto* m = M(h);
    if (layer_id < 0 || layer_id >= static_cast<int>(m->layers.size())) throw std::out_of_range("layer id");
    return flexflow_op_t{m->op(m->layers[layer_id])};
  });
}
flexflow_op_t flexflow_model_get_last_layer(flexflow_model_t h) {
  return guard(flexflow_op_t{nullptr}, [&] {
    auto* m = M(h);
    if (m->layers.empty()) throw std::out_of_range("model has no layers");
    return flexflow_op_t{m->op(m->layers.back())};
  });
}
flexflow_tensor_t flexflow_model_get_parameter_by_id(flexflow_model_t h, int layer_id) {
  // the reference leaves this unimplemented; here: the id-th weight tensor in
  // layer creation order
  return guard(nullT(), [&] {
    auto* m = M(h);
    int k = 0;
    for (int n : m->layers)
      for (auto const& w : m->cg.layer_weights(n))
        if (k++ == layer_id) return wrapT(m->wrap(w));
    throw std::out_of_range("parameter id");
  });
}
flexflow_perf_metrics_t flexflow_model_get_perf_metrics(flexflow_model_t h) {
  return guard(flexflow_perf_metrics_t{nullptr}, [&] {
    auto* m = M(h);
    auto* p = new RtMetrics();
    if (m->be) {
      const auto& mm = m->be->metrics();
      p->correct = mm.correct;
      p->all = mm.samples;
      p->loss = mm.loss_sum;
    }
    return flexflow_perf_metrics_t{p};
  });
}
bool flexflow_model_get_output_tensor_float(flexflow_model_t model, flexflow_tensor_t handle, float* data,
                                            bool get_gradients) {
  return flexflow_tensor_get_tensor_float(handle, model, data, get_gradients);
}

// ---- Tensor ----------------------------------------------------------------
flexflow_tensor_t flexflow_tensor_create(flexflow_model_t model, int num_dims, const int* dims,
                                         enum DataType data_type, bool create_grad) {
  return guard(nullT(), [&] {
    auto* m = M(model);
    if (m->be) throw std::runtime_error("tensors cannot be created after compile()");
    auto v = m->cg.create_input(ff::TensorShape{ints(dims, num_dims), dtype_of(data_type)}, create_grad);
    return wrapT(m->wrap(v));
  });
}
void flexflow_tensor_map(flexflow_model_t, flexflow_tensor_t, flexflow_op_t) {}
flexflow_tensor_t flexflow_constant_create(flexflow_model_t model, int num_dims, const int* dims, float value,
                                           enum DataType data_type) {
  return guard(nullT(), [&] {
    auto* m = M(model);
    if (m->be) throw std::runtime_error("tensors cannot be created after compile()");
    std::ostringstream init;
    init << R"({"type":"constant","value":)" << value << "}";
    auto v = m->cg.create_weight(ff::TensorShape{ints(dims, num_dims), dtype_of(data_type)}, init.str(), false);
    return wrapT(m->wrap(v));
  });
}
void flexflow_tensor_destroy(flexflow_tensor_t) {}  // tensors are owned by their model
void flexflow_tensor_inline_map(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t) {
  guard_void([&] { T(handle)->mapped = true; });
}
void flexflow_tensor_inline_unmap(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t) {
  guard_void([&] {
    auto* t = T(handle);
    if (!t->i32.empty()) {  // write an int32 view back into the float slot
      float* d = t->m->data(t, false);
      for (size_t i = 0; i < t->i32.size(); ++i) d[i] = static_cast<float>(t->i32[i]);
      t->i32.clear();
    }
    t->mapped = false;
  });
}
float* flexflow_tensor_get_raw_ptr_float(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t) {
  return guard(static_cast<float*>(nullptr), [&] {
    auto* t = T(handle);
    return t->m->data(t, false);
  });
}
int32_t* flexflow_tensor_get_raw_ptr_int32(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t) {
  return guard(static_cast<int32_t*>(nullptr), [&] {
    auto* t = T(handle);
    const float* d = t->m->data(t, false);
    t->i32.resize(static_cast<size_t>(t->numel()));
    for (size_t i = 0; i < t->i32.size(); ++i) t->i32[i] = static_cast<int32_t>(d[i]);
    return t->i32.data();
  });
}
int flexflow_tensor_get_num_dims(flexflow_tensor_t handle) {
  return guard(-1, [&] { return static_cast<int>(T(handle)->dims.size()); });
}
int flexflow_tensor_get_dim(flexflow_tensor_t handle, int legion_axis) {
  return guard(-1, [&] { return T(handle)->legion_dims.at(static_cast<size_t>(legion_axis)); });
}
int* flexflow_tensor_get_dims(flexflow_tensor_t handle) {
  return guard(static_cast<int*>(nullptr), [&] { return T(handle)->legion_dims.data(); });
}
int flexflow_tensor_get_data_type(flexflow_tensor_t handle) {
  return guard(-1, [&] { return dtype_enum(T(handle)->dtype); });
}
flexflow_op_t flexflow_tensor_get_owner_op(flexflow_tensor_t handle) {
  return guard(flexflow_op_t{nullptr}, [&] {
    auto* t = T(handle);
    if (t->v.node < 0) return flexflow_op_t{nullptr};
    const ff::OpType ty = t->m->cg.g.node(t->v.node).label.op.type;
    if (ty == ff::OpType::INPUT || ty == ff::OpType::WEIGHT) return flexflow_op_t{nullptr};
    return flexflow_op_t{t->m->op(t->v.node)};
  });
}
void flexflow_tensor_attach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t, void* raw_ptr,
                                    bool column_major) {
  guard_void([&] {
    auto* t = T(handle);
    if (column_major) throw std::invalid_argument("column-major attach is not supported");
    const int64_t n = t->numel();
    float* d = t->m->data(t, false);
    if (t->dtype == ff::DataType::INT32) {
      auto p = static_cast<const int32_t*>(raw_ptr);
      for (int64_t i = 0; i < n; ++i) d[i] = static_cast<float>(p[i]);
    } else if (t->dtype == ff::DataType::INT64) {
      auto p = static_cast<const int64_t*>(raw_ptr);
      for (int64_t i = 0; i < n; ++i) d[i] = static_cast<float>(p[i]);
    } else {
      std::memcpy(d, raw_ptr, sizeof(float) * static_cast<size_t>(n));
    }
    t->mapped = true;
  });
}
void flexflow_tensor_detach_raw_ptr(flexflow_tensor_t handle, flexflow_model_t, flexflow_config_t) {
  guard_void([&] { T(handle)->mapped = false; });
}
bool flexflow_tensor_is_mapped(flexflow_tensor_t handle) {
  return guard(false, [&] { return T(handle)->mapped; });
}
bool flexflow_tensor_set_tensor_float(flexflow_tensor_t handle, flexflow_model_t, int num_dim, int* dims,
                                      const float* data) {
  return guard(false, [&] { return copy_in(T(handle), data, count(num_dim, dims)); });
}
bool flexflow_tensor_get_tensor_float(flexflow_tensor_t handle, flexflow_model_t, float* data, bool get_gradients) {
  return guard(false, [&] {
    auto* t = T(handle);
    const float* d = t->m->data(t, get_gradients);
    if (!d) throw std::runtime_error("tensor has no gradient");
    std::memcpy(data, d, sizeof(float) * static_cast<size_t>(t->numel()));
    return true;
  });
}
bool flexflow_tensor_set_tensor_int(flexflow_tensor_t handle, flexflow_model_t, int num_dim, int* dims,
                                    const int* data) {
  return guard(false, [&] {
    auto* t = T(handle);
    const int64_t n = count(num_dim, dims);
    if (n != t->numel()) throw std::invalid_argument("tensor size mismatch");
    float* d = t->m->data(t, false);
    for (int64_t i = 0; i < n; ++i) d[i] = static_cast<float>(data[i]);
    return true;
  });
}
bool flexflow_tensor_get_tensor_int(flexflow_tensor_t handle, flexflow_model_t, int* data, bool get_gradients) {
  return guard(false, [&] {
    auto* t = T(handle);
    const float* d = t->m->data(t, get_gradients);
    if (!d) throw std::runtime_error("tensor has no gradient");
    for (int64_t i = 0; i < t->numel(); ++i) data[i] = static_cast<int>(d[i]);
    return true;
  });
}
bool flexflow_tensor_set_tensor_int64(flexflow_tensor_t handle, flexflow_model_t, int num_dim, int* dims,
                                      const int64_t* data, enum ParameterSyncType) {
  return guard(false, [&] {
    auto* t = T(handle);
    const int64_t n = count(num_dim, dims);
    if (n != t->numel()) throw std::invalid_argument("tensor size mismatch");
    float* d = t->m->data(t, false);
    for (int64_t i = 0; i < n; ++i) d[i] = static_cast<float>(data[i]);
    return true;
  });
}
bool flexflow_tensor_get_tensor_int64(flexflow_tensor_t handle, flexflow_model_t, int64_t* data,
                                      bool get_gradients) {
  return guard(false, [&] {
    auto* t = T(handle);
    const float* d = t->m->data(t, get_gradients);
    if (!d) throw std::runtime_error("tensor has no gradient");
    for (int64_t i = 0; i < t->numel(); ++i) data[i] = static_cast<int64_t>(d[i]);
    return true;
  });
}
bool flexflow_parameter_set_weights_float(flexflow_tensor_t handle, flexflow_model_t model, int num_dim, int* dims,
                                          const float* data) {
  return flexflow_tensor_set_tensor_float(handle, model, num_dim, dims, data);
}
bool flexflow_parameter_get_weights_float(flexflow_tensor_t handle, flexflow_model_t model, float* data) {
  return flexflow_tensor_get_tensor_float(handle, model, data, false);
}

// ---- Optimizers / initializers / metrics --------------------------------------
flexflow_sgd_optimizer_t flexflow_sgd_optimizer_create(flexflow_model_t, double lr, double momentum, bool nesterov,
                                                       double weight_decay) {
  auto* o = new RtOptimizer();
  o->o.kind = "sgd";
  o->o.lr = lr;
  o->o.momentum = momentum;
  o->o.nesterov = nesterov;
  o->o.weight_decay = weight_decay;
  return flexflow_sgd_optimizer_t{o};
}
void flexflow_sgd_optimizer_destroy(flexflow_sgd_optimizer_t h) { delete static_cast<RtOptimizer*>(h.impl); }
void flexflow_sgd_optimizer_set_lr(flexflow_sgd_optimizer_t h, double lr) {
  guard_void([&] {
    auto* o = impl<RtOptimizer>(h.impl, "optimizer");
    o->o.lr = lr;
    if (o->m) o->m->opt.lr = lr;
  });
}
flexflow_adam_optimizer_t flexflow_adam_optimizer_create(flexflow_model_t, double alpha, double beta1, double beta2,
                                                         double weight_decay, double epsilon) {
  auto* o = new RtOptimizer();
  o->o.kind = "adam";
  o->o.lr = alpha;
  o->o.beta1 = beta1;
  o->o.beta2 = beta2;
  o->o.weight_decay = weight_decay;
  o->o.epsilon = epsilon;
  return flexflow_adam_optimizer_t{o};
}
void flexflow_adam_optimizer_destroy(flexflow_adam_optimizer_t h) { delete static_cast<RtOptimizer*>(h.impl); }
void flexflow_adam_optimizer_set_lr(flexflow_adam_optimizer_t h, double lr) {
  guard_void([&] {
    auto* o = impl<RtOptimizer>(h.impl, "optimizer");
    o->o.lr = lr;
    if (o->m) o->m->opt.lr = lr;
  });
}

flexflow_initializer_t flexflow_initializer_create_null(void) { return flexflow_initializer_t{nullptr}; }
flexflow_glorot_uniform_initializer_t flexflow_glorot_uniform_initializer_create(int seed) {
  return flexflow_glorot_uniform_initializer_t{
      new RtInit{R"({"type":"glorot_uniform","seed":)" + std::to_string(seed) + "}"}};
}
void flexflow_glorot_uniform_initializer_destroy(flexflow_glorot_uniform_initializer_t h) {
  delete static_cast<RtInit*>(h.impl);
}
flexflow_zero_initializer_t flexflow_zero_initializer_create(void) {
  return flexflow_zero_initializer_t{new RtInit{R"({"type":"zero"})"}};
}
void flexflow_zero_initializer_destroy(flexflow_zero_initializer_t h) { delete static_cast<RtInit*>(h.impl); }
flexflow_uniform_initializer_t flexflow_uniform_initializer_create(int seed, float min, float max) {
  std::ostringstream s;
  s << R"({"type":"uniform","seed":)" << seed << R"(,"min":)" << min << R"(,"max":)" << max << "}";
  return flexflow_uniform_initializer_t{new RtInit{s.str()}};
}
void flexflow_uniform_initializer_destroy(flexflow_uniform_initializer_t h) { delete static_cast<RtInit*>(h.impl); }
flexflow_norm_initializer_t flexflow_norm_initializer_create(int seed, float mean, float stddev) {
  std::ostringstream s;
  s << R"({"type":"normal","seed":)" << seed << R"(,"mean":)" << mean << R"(,"stddev":)" << stddev << "}";
  return flexflow_norm_initializer_t{new RtInit{s.str()}};
}
void flexflow_norm_initializer_destroy(flexflow_norm_initializer_t h) { delete static_cast<RtInit*>(h.impl); }

void flexflow_per_metrics_destroy(flexflow_perf_metrics_t h) { delete static_cast<RtMetrics*>(h.impl); }
float flexflow_per_metrics_get_accuracy(flexflow_perf_metrics_t h) {
  return guard(0.f, [&] {
    auto* p = impl<RtMetrics>(h.impl, "perf metrics");
    return p->all ? static_cast<float>(p->correct) * 100.0f / static_cast<float>(p->all) : 0.f;
  });
}

// ---- example configs -------------------------------------------------------------
flexflow_net_config_t flexflow_net_config_create(void) { return flexflow_net_config_t{new RtNetConfig()}; }
void flexflow_net_config_destroy(flexflow_net_config_t h) { delete static_cast<RtNetConfig*>(h.impl); }
const char* flexflow_net_config_get_dataset_path(flexflow_net_config_t h) {
  return guard(static_cast<const char*>(nullptr),
               [&] { return impl<RtNetConfig>(h.impl, "net config")->dataset.c_str(); });
}
flexflow_dlrm_config_t flexflow_dlrm_config_create(void) { return flexflow_dlrm_config_t{new RtDLRMConfig()}; }
void flexflow_dlrm_config_destroy(flexflow_dlrm_config_t h) { delete static_cast<RtDLRMConfig*>(h.impl); }
#define DLRM(h) impl<RtDLRMConfig>((h).impl, "dlrm config")
const char* flexflow_dlrm_config_get_dataset_path(flexflow_dlrm_config_t h) {
  return guard(static_cast<const char*>(nullptr), [&] { return DLRM(h)->dataset.c_str(); });
}
const char* flexflow_dlrm_config_get_arch_interaction_op(flexflow_dlrm_config_t h) {
  return guard(static_cast<const char*>(nullptr), [&] { return DLRM(h)->interaction.c_str(); });
}
int flexflow_dlrm_config_get_sparse_feature_size(flexflow_dlrm_config_t h) {
  return guard(-1, [&] { return DLRM(h)->sparse_feature_size; });
}
int flexflow_dlrm_config_get_sigmoid_bot(flexflow_dlrm_config_t h) {
  return guard(-1, [&] { return DLRM(h)->sigmoid_bot; });
}
int flexflow_dlrm_config_get_sigmoid_top(flexflow_dlrm_config_t h) {
  return guard(-1, [&] { return DLRM(h)->sigmoid_top; });
}
int flexflow_dlrm_config_get_embedding_bag_size(flexflow_dlrm_config_t h) {
  return guard(-1, [&] { return DLRM(h)->embedding_bag_size; });
}
float flexflow_dlrm_config_get_loss_threshold(flexflow_dlrm_config_t h) {
  return guard(0.f, [&] { return DLRM(h)->loss_threshold; });
}
int* flexflow_dlrm_config_get_mlp_bot(flexflow_dlrm_config_t h) {
  return guard(static_cast<int*>(nullptr), [&] {
    auto* c = DLRM(h);
    c->out_bot = int_list(c->mlp_bot);
    return c->out_bot.data();
  });
}
int* flexflow_dlrm_config_get_mlp_top(flexflow_dlrm_config_t h) {
  return guard(static_cast<int*>(nullptr), [&] {
    auto* c = DLRM(h);
    c->out_top = int_list(c->mlp_top);
    return c->out_top.data();
  });
}
int* flexflow_dlrm_config_get_embedding_size(flexflow_dlrm_config_t h) {
  return guard(static_cast<int*>(nullptr), [&] {
    auto* c = DLRM(h);
    c->out_emb = int_list(c->embedding_size);
    return c->out_emb.data();
  });
}
#undef DLRM

// ---- SingleDataLoader ----------------------------------------------------------------
flexflow_single_dataloader_t flexflow_single_dataloader_create(flexflow_model_t ffmodel, flexflow_tensor_t input,
                                                               flexflow_tensor_t full_input, int num_samples,
                                                               enum DataType data_type) {
  return guard(flexflow_single_dataloader_t{nullptr}, [&] {
    auto* full = T(full_input);
    auto* m = M(ffmodel);
    const float* src = m->data(full, false);
    auto l = std::make_unique<RtLoader>();
    l->m = m;
    l->batch = T(input);
    l->num_samples = num_samples;
    l->sample = l->batch->numel() / std::max<int64_t>(1, l->batch->dims.empty() ? 1 : l->batch->dims[0]);
    if (full->numel() < num_samples * l->sample) throw std::invalid_argument("full input smaller than num_samples");
    l->load(src, DT_FLOAT, num_samples * l->sample);  // slots hold floats whatever the data type
    (void)data_type;
    return flexflow_single_dataloader_t{l.release()};
  });
}
flexflow_single_dataloader_t flexflow_single_dataloader_create2(flexflow_model_t ffmodel, flexflow_tensor_t input,
                                                                void* full_input_ptr, int num_samples,
                                                                enum DataType data_type) {
  return guard(flexflow_single_dataloader_t{nullptr}, [&] {
    auto l = std::make_unique<RtLoader>();
    l->m = M(ffmodel);
    l->batch = T(input);
    l->num_samples = num_samples;
    l->sample = l->batch->numel() / std::max<int64_t>(1, l->batch->dims.empty() ? 1 : l->batch->dims[0]);
    l->load(full_input_ptr, data_type, num_samples * l->sample);
    return flexflow_single_dataloader_t{l.release()};
  });
}
void flexflow_single_dataloader_destroy(flexflow_single_dataloader_t h) { delete static_cast<RtLoader*>(h.impl); }
void flexflow_single_dataloader_set_num_samples(flexflow_single_dataloader_t h, int samples) {
  guard_void([&] {
    auto* l = impl<RtLoader>(h.impl, "dataloader");
    if (static_cast<int64_t>(samples) * l->sample > static_cast<int64_t>(l->full.size()))
      throw std::invalid_argument("more samples than loaded");
    l->num_samples = samples;
  });
}
int flexflow_single_dataloader_get_num_samples(flexflow_single_dataloader_t h) {
  return guard(-1, [&] { return static_cast<int>(impl<RtLoader>(h.impl, "dataloader")->num_samples); });
}
void flexflow_single_dataloader_reset(flexflow_single_dataloader_t h) {
  guard_void([&] { impl<RtLoader>(h.impl, "dataloader")->next = 0; });
}
void flexflow_single_dataloader_next_batch(flexflow_single_dataloader_t h, flexflow_model_t) {
  guard_void([&] { impl<RtLoader>(h.impl, "dataloader")->next_batch(); });
}
void flowflow_single_dataloader_next_batch(flexflow_single_dataloader_t h, flexflow_model_t m) {
  flexflow_single_dataloader_next_batch(h, m);
}

// ---- timing / tracing --------------------------------------------------------------
double flexflow_get_current_time(flexflow_config_t) { return now_us(); }
void flexflow_begin_trace(flexflow_config_t, int) {}
void flexflow_end_trace(flexflow_config_t, int) {}

// ---- Op ------------------------------------------------------------------------------
#define OPH(h) impl<RtOp>((h).impl, "op")
int flexflow_op_get_num_parameters(flexflow_op_t h) {
  return guard(-1, [&] {
    auto* o = OPH(h);
    return static_cast<int>(o->m->cg.layer_weights(o->node).size());
  });
}
flexflow_tensor_t flexflow_op_get_parameter_by_id(flexflow_op_t h, int id) {
  return guard(nullT(), [&] {
    auto* o = OPH(h);
    return wrapT(o->m->wrap(o->m->cg.layer_weights(o->node).at(static_cast<size_t>(id))));
  });
}
int flexflow_op_get_num_inputs(flexflow_op_t h) {
  return guard(-1, [&] {
    auto* o = OPH(h);
    return static_cast<int>(o->m->cg.layer_data_inputs(o->node).size());
  });
}
flexflow_tensor_t flexflow_op_get_input_by_id(flexflow_op_t h, int id) {
  return guard(nullT(), [&] {
    auto* o = OPH(h);
    return wrapT(o->m->wrap(o->m->cg.layer_data_inputs(o->node).at(static_cast<size_t>(id))));
  });
}
int flexflow_op_get_num_outputs(flexflow_op_t h) {
  return guard(-1, [&] {
    auto* o = OPH(h);
    return static_cast<int>(o->m->cg.g.node(o->node).outputs.size());
  });
}
flexflow_tensor_t flexflow_op_get_output_by_id(flexflow_op_t h, int id) {
  return guard(nullT(), [&] {
    auto* o = OPH(h);
    if (id < 0 || id >= static_cast<int>(o->m->cg.g.node(o->node).outputs.size())) throw std::out_of_range("output id");
    return wrapT(o->m->wrap(ff::ValueRef{o->node, id}));
  });
}
void flexflow_op_init(flexflow_op_t h, flexflow_model_t) {
  guard_void([&] { (void)OPH(h); });
}
void flexflow_op_forward(flexflow_op_t h, flexflow_model_t) {
  guard_void([&] {
    auto* o = OPH(h);
    if (!o->m->be) throw std::runtime_error("op forward before compile()");
    o->m->be->forward_layer(o->node);
  });
}
#undef OPH

// ---- task entry points ----------------------------------------------------------------
void register_c_custom_tasks(void) {}
void begin_flexflow_task(int argc, char** argv) {
  g_args.clear();
  for (int i = 0; i < argc; ++i) g_args.emplace_back(argv[i] ? argv[i] : "");
}
void finish_flexflow_task(void) { g_args.clear(); }

}  // extern "C"
