// C ABI over the ffcore library (see flexflow_c.h).
#include "flexflow_c.h"

#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "ff/computation_graph.h"
#include "ff/models.h"
#include "ff/search.h"

struct flexflow_computation_graph_s {
  ff::ComputationGraph cg;
};

struct flexflow_search_result_s {
  ff::SearchResult r;
  ff::ComputationGraph cg;
};

namespace {

thread_local std::string g_last_error;

flexflow_error_t fail(flexflow_error_t code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

template <typename F>
flexflow_error_t guarded(F&& f) {
  try {
    f();
    return FLEXFLOW_OK;
  } catch (const ff::FFError& e) {
    return fail(FLEXFLOW_ERROR_SHAPE, e.what());
  } catch (const std::invalid_argument& e) {
    return fail(FLEXFLOW_ERROR_INVALID_ARGUMENT, e.what());
  } catch (const std::exception& e) {
    return fail(FLEXFLOW_ERROR_INTERNAL, e.what());
  }
}

char* dup(const std::string& s) {
  char* p = static_cast<char*>(std::malloc(s.size() + 1));
  std::memcpy(p, s.c_str(), s.size() + 1);
  return p;
}

std::string nm(const char* s) { return s ? std::string(s) : std::string(); }

ff::ValueRef ref(flexflow_tensor_t t) { return ff::ValueRef{t.node, t.idx}; }
flexflow_tensor_t tens(ff::ValueRef v) { return flexflow_tensor_t{v.node, v.idx}; }

ff::Activation act(flexflow_activation_t a) { return static_cast<ff::Activation>(static_cast<int>(a)); }

#define CHECK_ARG(cond, msg) \
  if (!(cond)) return fail(FLEXFLOW_ERROR_INVALID_ARGUMENT, msg)

flexflow_error_t unary(flexflow_computation_graph_t cg, ff::OpType t, flexflow_tensor_t x, const char* name,
                       flexflow_tensor_t* out, double* scalar = nullptr) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    std::optional<double> s;
    if (scalar) s = *scalar;
    *out = tens(cg->cg.unary(t, ref(x), nm(name), s));
  });
}

flexflow_error_t binary(flexflow_computation_graph_t cg, ff::OpType t, flexflow_tensor_t a, flexflow_tensor_t b,
                        const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.binary(t, ref(a), ref(b), nm(name))); });
}

}  // namespace

extern "C" {

const char* flexflow_last_error(void) { return g_last_error.c_str(); }
void flexflow_free(void* p) { std::free(p); }
const char* flexflow_version(void) { return "flexflow-train-mi355x 0.1 (gfx950)"; }

// ---------------------------------------------------------------- graph
flexflow_error_t flexflow_computation_graph_create(flexflow_computation_graph_t* out) {
  CHECK_ARG(out, "null out");
  *out = new flexflow_computation_graph_s();
  return FLEXFLOW_OK;
}

flexflow_error_t flexflow_computation_graph_destroy(flexflow_computation_graph_t cg) {
  delete cg;
  return FLEXFLOW_OK;
}

flexflow_error_t flexflow_computation_graph_serialize_to_buf(flexflow_computation_graph_t cg, char** out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = dup(cg->cg.to_json().dump()); });
}

flexflow_error_t flexflow_computation_graph_deserialize_from_buf(const char* buf, flexflow_computation_graph_t* out) {
  CHECK_ARG(buf && out, "null argument");
  return guarded([&] {
    auto* g = new flexflow_computation_graph_s();
    try {
      g->cg = ff::ComputationGraph::from_json(ff::Json::parse(buf));
    } catch (...) {
      delete g;
      throw;
    }
    *out = g;
  });
}

flexflow_error_t flexflow_computation_graph_serialize_to_file(flexflow_computation_graph_t cg, const char* path) {
  CHECK_ARG(cg && path, "null argument");
  std::ofstream f(path);
  if (!f) return fail(FLEXFLOW_ERROR_IO, std::string("cannot write ") + path);
  return guarded([&] { f << cg->cg.to_json().dump(); });
}

flexflow_error_t flexflow_computation_graph_deserialize_from_file(const char* path,
                                                                  flexflow_computation_graph_t* out) {
  CHECK_ARG(path && out, "null argument");
  std::ifstream f(path);
  if (!f) return fail(FLEXFLOW_ERROR_IO, std::string("cannot read ") + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return flexflow_computation_graph_deserialize_from_buf(ss.str().c_str(), out);
}

flexflow_error_t flexflow_computation_graph_as_dot(flexflow_computation_graph_t cg, char** out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = dup(cg->cg.as_dot()); });
}

flexflow_error_t flexflow_computation_graph_num_layers(flexflow_computation_graph_t cg, int* out) {
  CHECK_ARG(cg && out, "null argument");
  *out = static_cast<int>(cg->cg.g.node_ids().size());
  return FLEXFLOW_OK;
}

flexflow_error_t flexflow_computation_graph_from_model(const char* name, flexflow_computation_graph_t* out) {
  CHECK_ARG(name && out, "null argument");
  return guarded([&] {
    auto* g = new flexflow_computation_graph_s();
    try {
      g->cg = ff::get_model_computation_graph(name, ff::Json::object());
    } catch (...) {
      delete g;
      throw;
    }
    *out = g;
  });
}

// -------------------------------------------------------------- tensors
flexflow_error_t flexflow_tensor_create(flexflow_computation_graph_t cg, int num_dims, const int64_t* dims,
                                        flexflow_datatype_t dtype, bool create_grad, const char* name,
                                        flexflow_tensor_t* out) {
  CHECK_ARG(cg && out && (num_dims == 0 || dims), "null argument");
  CHECK_ARG(num_dims >= 0 && num_dims <= 8, "num_dims out of range");
  return guarded([&] {
    ff::TensorShape s;
    s.dims.assign(dims, dims + num_dims);
    s.dtype = static_cast<ff::DataType>(static_cast<int>(dtype));
    *out = tens(cg->cg.create_input(s, create_grad, nm(name)));
  });
}

flexflow_error_t flexflow_tensor_get_num_dims(flexflow_computation_graph_t cg, flexflow_tensor_t t, int* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = cg->cg.shape(ref(t)).num_dims(); });
}

flexflow_error_t flexflow_tensor_get_dims(flexflow_computation_graph_t cg, flexflow_tensor_t t, int64_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    auto const& s = cg->cg.shape(ref(t));
    for (int i = 0; i < s.num_dims(); ++i) out[i] = s.dims[i];
  });
}

flexflow_error_t flexflow_tensor_get_datatype(flexflow_computation_graph_t cg, flexflow_tensor_t t,
                                              flexflow_datatype_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = static_cast<flexflow_datatype_t>(static_cast<int>(cg->cg.shape(ref(t)).dtype)); });
}

// ------------------------------------------------------------ operators
flexflow_error_t flexflow_computation_graph_add_op(flexflow_computation_graph_t cg, const char* attrs_json,
                                                   int num_inputs, const flexflow_tensor_t* inputs,
                                                   const char* name, int max_outputs, flexflow_tensor_t* outputs,
                                                   int* num_outputs) {
  CHECK_ARG(cg && attrs_json && (num_inputs == 0 || inputs), "null argument");
  return guarded([&] {
    auto j = ff::Json::parse(attrs_json);
    ff::Json wrapped = j;
    if (!j.contains("attrs")) {  // flat form {"op_type": ..., key: value, ...}
      wrapped = ff::Json::object();
      ff::Json attrs = ff::Json::object();
      for (auto const& kv : j.as_object()) {
        if (kv.first == "op_type") wrapped["op_type"] = kv.second;
        else attrs[kv.first] = kv.second;
      }
      wrapped["attrs"] = attrs;
    }
    ff::OpAttrs op = ff::normalize_attrs(ff::OpAttrs::from_json(wrapped));
    std::vector<ff::ValueRef> ins;
    for (int i = 0; i < num_inputs; ++i) ins.push_back(ref(inputs[i]));
    auto outs = cg->cg.add_layer(op, ins, nm(name));
    if (num_outputs) *num_outputs = static_cast<int>(outs.size());
    for (int i = 0; i < static_cast<int>(outs.size()) && i < max_outputs && outputs; ++i) outputs[i] = tens(outs[i]);
  });
}

flexflow_error_t flexflow_computation_graph_add_op_dense(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                         int64_t out_dim, flexflow_activation_t a, bool use_bias,
                                                         const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.dense(ref(x), out_dim, act(a), use_bias, nm(name))); });
}

#define FF_UNARY(fn, T)                                                                                  \
  flexflow_error_t fn(flexflow_computation_graph_t cg, flexflow_tensor_t x, const char* name,            \
                      flexflow_tensor_t* out) {                                                          \
    return unary(cg, ff::OpType::T, x, name, out);                                                       \
  }
FF_UNARY(flexflow_computation_graph_add_op_relu, RELU)
FF_UNARY(flexflow_computation_graph_add_op_gelu, GELU)
FF_UNARY(flexflow_computation_graph_add_op_sigmoid, SIGMOID)
FF_UNARY(flexflow_computation_graph_add_op_tanh, TANH)
FF_UNARY(flexflow_computation_graph_add_op_exp, EXP)
FF_UNARY(flexflow_computation_graph_add_op_identity, IDENTITY)
FF_UNARY(flexflow_computation_graph_add_op_rsqrt, RSQRT)
#undef FF_UNARY

flexflow_error_t flexflow_computation_graph_add_op_scalar_multiply(flexflow_computation_graph_t cg,
                                                                   flexflow_tensor_t x, double s, const char* name,
                                                                   flexflow_tensor_t* out) {
  return unary(cg, ff::OpType::SCALAR_MULTIPLY, x, name, out, &s);
}

flexflow_error_t flexflow_computation_graph_add_op_scalar_add(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                              double s, const char* name, flexflow_tensor_t* out) {
  return unary(cg, ff::OpType::SCALAR_ADD, x, name, out, &s);
}

#define FF_BINARY(fn, T)                                                                                 \
  flexflow_error_t fn(flexflow_computation_graph_t cg, flexflow_tensor_t a, flexflow_tensor_t b,         \
                      const char* name, flexflow_tensor_t* out) {                                        \
    return binary(cg, ff::OpType::T, a, b, name, out);                                                   \
  }
FF_BINARY(flexflow_computation_graph_add_op_add, EW_ADD)
FF_BINARY(flexflow_computation_graph_add_op_subtract, EW_SUB)
FF_BINARY(flexflow_computation_graph_add_op_multiply, EW_MUL)
FF_BINARY(flexflow_computation_graph_add_op_divide, EW_DIV)
#undef FF_BINARY

flexflow_error_t flexflow_computation_graph_add_op_softmax(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                           int dim, const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.softmax(ref(x), dim, nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_layer_norm(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                              int num_axes, const int64_t* axes, bool affine,
                                                              double eps, const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out && (num_axes == 0 || axes), "null argument");
  return guarded([&] {
    *out = tens(cg->cg.layer_norm(ref(x), std::vector<int64_t>(axes, axes + num_axes), affine, eps, nm(name)));
  });
}

flexflow_error_t flexflow_computation_graph_add_op_batch_norm(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                              bool relu, const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.batch_norm(ref(x), relu, nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_embedding(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                             int64_t num_entries, int64_t out_dim, const char* aggr,
                                                             const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    *out = tens(cg->cg.embedding(ref(x), num_entries, out_dim, aggr ? aggr : "none", ff::DataType::FLOAT,
                                 nm(name)));
  });
}

flexflow_error_t flexflow_computation_graph_add_op_batch_matmul(flexflow_computation_graph_t cg, flexflow_tensor_t a,
                                                                flexflow_tensor_t b, const char* name,
                                                                flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.batch_matmul(ref(a), ref(b), nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_conv2d(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                          int64_t out_channels, int kernel_h, int kernel_w,
                                                          int stride_h, int stride_w, int padding_h, int padding_w,
                                                          flexflow_activation_t a, int groups, bool use_bias,
                                                          const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    *out = tens(cg->cg.conv2d(ref(x), out_channels, kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                              act(a), groups, use_bias, nm(name)));
  });
}

flexflow_error_t flexflow_computation_graph_add_op_pool2d(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                          int kernel_h, int kernel_w, int stride_h, int stride_w,
                                                          int padding_h, int padding_w, const char* pool_type,
                                                          const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    *out = tens(cg->cg.pool2d(ref(x), kernel_h, kernel_w, stride_h, stride_w, padding_h, padding_w,
                              pool_type ? pool_type : "max", ff::Activation::NONE, nm(name)));
  });
}

flexflow_error_t flexflow_computation_graph_add_op_flat(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                        const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.flat(ref(x), nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_reshape(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                           int num_dims, const int64_t* shape, const char* name,
                                                           flexflow_tensor_t* out) {
  CHECK_ARG(cg && out && shape, "null argument");
  return guarded([&] { *out = tens(cg->cg.reshape(ref(x), std::vector<int64_t>(shape, shape + num_dims), nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_transpose(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                             int num_dims, const int64_t* perm, const char* name,
                                                             flexflow_tensor_t* out) {
  CHECK_ARG(cg && out && perm, "null argument");
  return guarded([&] { *out = tens(cg->cg.transpose(ref(x), std::vector<int64_t>(perm, perm + num_dims), nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_op_concat(flexflow_computation_graph_t cg, int num_inputs,
                                                          const flexflow_tensor_t* xs, int axis, const char* name,
                                                          flexflow_tensor_t* out) {
  CHECK_ARG(cg && out && xs && num_inputs > 0, "null argument");
  return guarded([&] {
    std::vector<ff::ValueRef> v;
    for (int i = 0; i < num_inputs; ++i) v.push_back(ref(xs[i]));
    *out = tens(cg->cg.concat(v, axis, nm(name)));
  });
}

flexflow_error_t flexflow_computation_graph_add_op_split(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                         int num_splits, const int64_t* sizes, int axis,
                                                         const char* name, flexflow_tensor_t* outs) {
  CHECK_ARG(cg && outs && sizes && num_splits > 0, "null argument");
  return guarded([&] {
    auto r = cg->cg.split(ref(x), std::vector<int64_t>(sizes, sizes + num_splits), axis, nm(name));
    for (size_t i = 0; i < r.size(); ++i) outs[i] = tens(r[i]);
  });
}

flexflow_error_t flexflow_computation_graph_add_op_dropout(flexflow_computation_graph_t cg, flexflow_tensor_t x,
                                                           double rate, int64_t seed, const char* name,
                                                           flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] { *out = tens(cg->cg.dropout(ref(x), rate, seed, nm(name))); });
}

flexflow_error_t flexflow_computation_graph_add_multihead_attention(flexflow_computation_graph_t cg,
                                                                    flexflow_tensor_t q, flexflow_tensor_t k,
                                                                    flexflow_tensor_t v, int64_t embed_dim,
                                                                    int64_t num_heads, int64_t kdim, int64_t vdim,
                                                                    double dropout, bool bias, bool causal,
                                                                    const char* name, flexflow_tensor_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    *out = tens(cg->cg.multihead_attention(ref(q), ref(k), ref(v), embed_dim, num_heads, kdim, vdim, dropout, bias,
                                           causal, nm(name)));
  });
}

// ------------------------------------------------------------- compiler
flexflow_error_t flexflow_computation_graph_optimize(flexflow_computation_graph_t cg, const char* machine_json,
                                                     const char* search_json, flexflow_search_result_t* out) {
  CHECK_ARG(cg && out, "null argument");
  return guarded([&] {
    ff::Json mj = (machine_json && *machine_json) ? ff::Json::parse(machine_json) : ff::Json::object();
    ff::Json sj = (search_json && *search_json) ? ff::Json::parse(search_json) : ff::Json::object();
    ff::MachineSpecification spec = ff::MachineSpecification::from_json(mj);
    if (!sj.contains("world")) sj["world"] = static_cast<int64_t>(spec.num_nodes * spec.num_gpus_per_node);
    ff::SearchConfig cfg = ff::search_config_from_json(sj);
    ff::CostModel cm(spec);
    std::string algo = sj.contains("algorithm") ? sj.at("algorithm").as_string() : std::string("unity");
    auto* res = new flexflow_search_result_s();
    res->cg = cg->cg;
    try {
      if (algo == "mcmc") {
        res->r = ff::mcmc_search(cg->cg, cm, cfg);
      } else if (algo == "data_parallel") {
        auto st = ff::data_parallel_strategy(cg->cg, cfg.world);
        auto L = ff::lower_strategy(cg->cg, st, cfg.world);
        res->r.algorithm = "data_parallel";
        res->r.pcg = L.pcg;
        res->r.strategy = st;
        res->r.cost = res->r.data_parallel_cost = ff::evaluate_strategy(cg->cg, st, cm, cfg.sim, cfg.world);
      } else if (algo == "unity") {
        res->r = ff::graph_optimize(cg->cg, cm, cfg);
      } else {
        throw std::invalid_argument("unknown search algorithm '" + algo + "'");
      }
    } catch (...) {
      delete res;
      throw;
    }
    *out = res;
  });
}

flexflow_error_t flexflow_search_result_destroy(flexflow_search_result_t r) {
  delete r;
  return FLEXFLOW_OK;
}

flexflow_error_t flexflow_search_result_get_cost(flexflow_search_result_t r, double* seconds,
                                                 double* data_parallel_seconds) {
  CHECK_ARG(r, "null result");
  if (seconds) *seconds = r->r.cost;
  if (data_parallel_seconds) *data_parallel_seconds = r->r.data_parallel_cost;
  return FLEXFLOW_OK;
}

flexflow_error_t flexflow_search_result_get_report_json(flexflow_search_result_t r, char** out) {
  CHECK_ARG(r && out, "null argument");
  return guarded([&] { *out = dup(r->r.to_json(&r->cg).dump()); });
}

flexflow_error_t flexflow_search_result_get_parallel_computation_graph_json(flexflow_search_result_t r, char** out) {
  CHECK_ARG(r && out, "null argument");
  return guarded([&] { *out = dup(r->r.pcg.to_json().dump()); });
}

flexflow_error_t flexflow_search_result_get_parallel_layer_for_layer(flexflow_search_result_t r, int cg_node,
                                                                    int* pcg_node) {
  CHECK_ARG(r && pcg_node, "null argument");
  return guarded([&] {
    *pcg_node = -1;
    const std::string& name = r->cg.g.node(cg_node).label.name;
    for (int id : r->r.pcg.g.node_ids())
      if (!name.empty() && r->r.pcg.g.node(id).label.name == name) {
        *pcg_node = id;
        break;
      }
  });
}

}  // extern "C"
