#include "ff/computation_graph.h"

#include <algorithm>
#include <cctype>
#include <sstream>

namespace ff {

std::string default_initializer(OpType op, const std::string& w) {
  if (w == "bias" || w == "beta" || w == "input_bias" || w == "output_bias") return R"({"type":"zero"})";
  if (w == "gamma") return R"({"type":"constant","value":1.0})";
  if (op == OpType::EMBEDDING) return R"({"type":"normal","seed":0,"mean":0.0,"stddev":0.02})";
  return R"({"type":"glorot_uniform","seed":0})";
}

static std::string lower(std::string s) {
  for (auto& c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

// ===========================================================================
// ComputationGraph
std::string ComputationGraph::unique_name(const std::string& base, OpType t) {
  if (!base.empty()) return base;
  return lower(to_string(t)) + "_" + std::to_string(name_counter_++);
}

ValueRef ComputationGraph::create_input(const TensorShape& shape, bool create_grad, const std::string& name) {
  OpAttrs a(OpType::INPUT);
  a.set("dims", shape.dims).set("data_type", to_string(shape.dtype));
  a = normalize_attrs(a);
  int id = g.add_node(LayerAttrs{a, unique_name(name, OpType::INPUT)}, {},
                      {TensorAttrs{shape, create_grad, ""}});
  return {id, 0};
}

void ComputationGraph::set_input_replicated(int node) {
  auto& n = g.node(node);
  if (n.label.op.type != OpType::INPUT) throw FFError("set_input_replicated: not an INPUT node");
  n.label.op.set("replicated", true);
}

ValueRef ComputationGraph::create_weight(const TensorShape& shape, const std::string& init, bool create_grad,
                                         const std::string& name) {
  OpAttrs a(OpType::WEIGHT);
  a.set("dims", shape.dims).set("data_type", to_string(shape.dtype)).set("initializer", init);
  a = normalize_attrs(a);
  int id = g.add_node(LayerAttrs{a, unique_name(name, OpType::WEIGHT)}, {},
                      {TensorAttrs{shape, create_grad, init}});
  return {id, 0};
}

std::vector<ValueRef> ComputationGraph::add_layer(const OpAttrs& op_in, const std::vector<ValueRef>& inputs,
                                                  const std::string& name,
                                                  const std::vector<std::string>& inits) {
  OpAttrs op = normalize_attrs(op_in);
  std::vector<TensorShape> in_shapes;
  for (auto const& v : inputs) in_shapes.push_back(shape(v));
  auto wshapes = infer_weight_shapes(op, in_shapes);
  auto wnames = weight_names(op);
  std::string lname = unique_name(name, op.type);
  std::vector<ValueRef> weights;
  for (size_t i = 0; i < wshapes.size(); ++i) {
    std::string init = (i < inits.size() && !inits[i].empty()) ? inits[i] : default_initializer(op.type, wnames[i]);
    weights.push_back(create_weight(wshapes[i], init, true, lname + "." + wnames[i]));
  }
  return add_layer_with_weights(op, inputs, weights, lname);
}

std::vector<ValueRef> ComputationGraph::add_layer_with_weights(const OpAttrs& op_in,
                                                               const std::vector<ValueRef>& inputs,
                                                               const std::vector<ValueRef>& weights,
                                                               const std::string& name) {
  OpAttrs op = normalize_attrs(op_in);
  std::vector<TensorShape> in_shapes;
  for (auto const& v : inputs) in_shapes.push_back(shape(v));
  auto wshapes = infer_weight_shapes(op, in_shapes);
  if (wshapes.size() != weights.size())
    throw FFError(to_string(op.type) + ": expected " + std::to_string(wshapes.size()) + " weights");
  for (size_t i = 0; i < weights.size(); ++i)
    if (shape(weights[i]) != wshapes[i])
      throw FFError(to_string(op.type) + ": weight " + std::to_string(i) + " has shape " +
                    shape(weights[i]).str() + ", expected " + wshapes[i].str());
  auto outs = infer_output_shapes(op, in_shapes);
  std::vector<TensorAttrs> out_attrs;
  for (auto const& s : outs) {
    bool grad = s.dtype == DataType::FLOAT || s.dtype == DataType::HALF || s.dtype == DataType::BFLOAT16 ||
                s.dtype == DataType::DOUBLE;
    out_attrs.push_back(TensorAttrs{s, grad, ""});
  }
  std::vector<ValueRef> all = inputs;
  all.insert(all.end(), weights.begin(), weights.end());
  int id = g.add_node(LayerAttrs{op, unique_name(name, op.type)}, all, out_attrs);
  std::vector<ValueRef> r;
  for (size_t i = 0; i < outs.size(); ++i) r.push_back({id, static_cast<int>(i)});
  return r;
}

ValueRef ComputationGraph::dense(ValueRef x, int64_t out_dim, Activation act, bool use_bias,
                                 const std::string& name, const std::string& kinit, const std::string& binit) {
  OpAttrs a = make_linear(out_dim, use_bias, act);
  return add_layer(a, {x}, name, {kinit, binit})[0];
}

ValueRef ComputationGraph::conv2d(ValueRef x, int64_t oc, int kh, int kw, int sh, int sw, int ph, int pw,
                                  Activation act, int groups, bool use_bias, const std::string& name) {
  OpAttrs a(OpType::CONV2D);
  a.set("out_channels", oc).set("kernel_h", kh).set("kernel_w", kw).set("stride_h", sh).set("stride_w", sw);
  a.set("padding_h", ph).set("padding_w", pw).set("groups", groups).set("activation", to_string(act));
  a.set("use_bias", use_bias);
  return add_layer(a, {x}, name)[0];
}

ValueRef ComputationGraph::pool2d(ValueRef x, int kh, int kw, int sh, int sw, int ph, int pw,
                                  const std::string& pool_type, Activation act, const std::string& name) {
  OpAttrs a(OpType::POOL2D);
  a.set("kernel_h", kh).set("kernel_w", kw).set("stride_h", sh).set("stride_w", sw);
  a.set("padding_h", ph).set("padding_w", pw).set("pool_type", pool_type).set("activation", to_string(act));
  return add_layer(a, {x}, name)[0];
}

ValueRef ComputationGraph::embedding(ValueRef x, int64_t n, int64_t d, const std::string& aggr, DataType dt,
                                     const std::string& name, const std::string& kinit) {
  OpAttrs a(OpType::EMBEDDING);
  a.set("num_entries", n).set("out_channels", d).set("aggr", aggr).set("data_type", to_string(dt));
  return add_layer(a, {x}, name, {kinit})[0];
}

ValueRef ComputationGraph::multihead_attention(ValueRef q, ValueRef k, ValueRef v, int64_t embed_dim,
                                               int64_t num_heads, int64_t kdim, int64_t vdim, double dropout,
                                               bool bias, bool causal, const std::string& name) {
  OpAttrs a(OpType::MULTIHEAD_ATTENTION);
  a.set("embed_dim", embed_dim).set("num_heads", num_heads).set("kdim", kdim).set("vdim", vdim);
  a.set("dropout", dropout).set("bias", bias).set("causal", causal);
  return add_layer(a, {q, k, v}, name)[0];
}

ValueRef ComputationGraph::layer_norm(ValueRef x, const std::vector<int64_t>& axes, bool affine, double eps,
                                      const std::string& name) {
  OpAttrs a(OpType::LAYERNORM);
  a.set("axes", axes).set("elementwise_affine", affine).set("eps", eps);
  return add_layer(a, {x}, name)[0];
}

ValueRef ComputationGraph::batch_norm(ValueRef x, bool relu, const std::string& name) {
  OpAttrs a(OpType::BATCHNORM);
  a.set("relu", relu);
  return add_layer(a, {x}, name)[0];
}

ValueRef ComputationGraph::softmax(ValueRef x, int dim, const std::string& name) {
  return add_layer(OpAttrs(OpType::SOFTMAX).set("dim", dim), {x}, name)[0];
}

ValueRef ComputationGraph::unary(OpType t, ValueRef x, const std::string& name, std::optional<double> scalar) {
  OpAttrs a(t);
  if (scalar) {
    if (t == OpType::POW) a.set("exponent", *scalar);
    else if (t == OpType::ELU || t == OpType::LEAKYRELU) a.set("alpha", *scalar);
    else a.set("scalar", *scalar);
  }
  return add_layer(a, {x}, name)[0];
}

ValueRef ComputationGraph::binary(OpType t, ValueRef x, ValueRef y, const std::string& name) {
  return add_layer(OpAttrs(t), {x, y}, name)[0];
}

ValueRef ComputationGraph::batch_matmul(ValueRef x, ValueRef y, const std::string& name) {
  return add_layer(OpAttrs(OpType::BATCHMATMUL), {x, y}, name)[0];
}

ValueRef ComputationGraph::concat(const std::vector<ValueRef>& xs, int axis, const std::string& name) {
  return add_layer(OpAttrs(OpType::CONCAT).set("axis", axis), xs, name)[0];
}

std::vector<ValueRef> ComputationGraph::split(ValueRef x, const std::vector<int64_t>& sizes, int axis,
                                              const std::string& name) {
  return add_layer(OpAttrs(OpType::SPLIT).set("axis", axis).set("splits", sizes), {x}, name);
}

ValueRef ComputationGraph::flat(ValueRef x, const std::string& name) {
  return add_layer(OpAttrs(OpType::FLAT), {x}, name)[0];
}

ValueRef ComputationGraph::reshape(ValueRef x, const std::vector<int64_t>& s, const std::string& name) {
  return add_layer(OpAttrs(OpType::RESHAPE).set("shape", s), {x}, name)[0];
}

ValueRef ComputationGraph::transpose(ValueRef x, const std::vector<int64_t>& perm, const std::string& name) {
  return add_layer(OpAttrs(OpType::TRANSPOSE).set("perm", perm), {x}, name)[0];
}

ValueRef ComputationGraph::reverse(ValueRef x, int axis, const std::string& name) {
  return add_layer(OpAttrs(OpType::REVERSE).set("axis", axis), {x}, name)[0];
}

ValueRef ComputationGraph::gather(ValueRef x, ValueRef idx, int dim, const std::string& name) {
  return add_layer(OpAttrs(OpType::GATHER).set("dim", dim), {x, idx}, name)[0];
}

ValueRef ComputationGraph::dropout(ValueRef x, double rate, int64_t seed, const std::string& name) {
  return add_layer(OpAttrs(OpType::DROPOUT).set("rate", rate).set("seed", seed), {x}, name)[0];
}

ValueRef ComputationGraph::cast(ValueRef x, DataType dt, const std::string& name) {
  return add_layer(OpAttrs(OpType::CAST).set("dtype", to_string(dt)), {x}, name)[0];
}

ValueRef ComputationGraph::reduce(OpType t, ValueRef x, const std::vector<int64_t>& axes, bool keepdims,
                                  const std::string& name) {
  return add_layer(OpAttrs(t).set("axes", axes).set("keepdims", keepdims), {x}, name)[0];
}

std::vector<ValueRef> ComputationGraph::top_k(ValueRef x, int k, bool sorted, const std::string& name) {
  return add_layer(OpAttrs(OpType::TOPK).set("k", k).set("sorted", sorted), {x}, name);
}

std::vector<ValueRef> ComputationGraph::layer_weights(int node) const {
  auto const& n = g.node(node);
  int nw = (n.label.op.type == OpType::INPUT || n.label.op.type == OpType::WEIGHT) ? 0 : num_weights(n.label.op);
  return std::vector<ValueRef>(n.inputs.end() - nw, n.inputs.end());
}

std::vector<ValueRef> ComputationGraph::layer_data_inputs(int node) const {
  auto const& n = g.node(node);
  int nw = (n.label.op.type == OpType::INPUT || n.label.op.type == OpType::WEIGHT) ? 0 : num_weights(n.label.op);
  return std::vector<ValueRef>(n.inputs.begin(), n.inputs.end() - nw);
}

std::optional<int> ComputationGraph::find_layer(const std::string& name) const {
  for (int id : g.node_ids())
    if (g.node(id).label.name == name) return id;
  return std::nullopt;
}

static Json value_ref_json(const ValueRef& v) { return Json(std::vector<int64_t>{v.node, v.idx}); }
static ValueRef value_ref_from(const Json& j) {
  auto xs = j.as_int_vector();
  return {static_cast<int>(xs.at(0)), static_cast<int>(xs.at(1))};
}

Json ComputationGraph::to_json() const {
  Json j = Json::object();
  j["format"] = "ffmi355x.computation_graph.v1";
  Json layers = Json::array();
  for (int id : g.topo_order()) {
    auto const& n = g.node(id);
    Json l = Json::object();
    l["id"] = id;
    l["name"] = n.label.name;
    l["op"] = n.label.op.to_json();
    Json ins = Json::array();
    for (auto const& v : n.inputs) ins.push_back(value_ref_json(v));
    l["inputs"] = ins;
    Json outs = Json::array();
    for (auto const& t : n.outputs) {
      Json o = Json::object();
      o["shape"] = t.shape.to_json();
      o["create_grad"] = t.create_grad;
      if (!t.initializer.empty()) o["initializer"] = Json::parse(t.initializer);
      outs.push_back(o);
    }
    l["outputs"] = outs;
    layers.push_back(l);
  }
  j["layers"] = layers;
  return j;
}

ComputationGraph ComputationGraph::from_json(const Json& j) {
  ComputationGraph cg;
  for (auto const& l : j.at("layers").as_array()) {
    std::vector<ValueRef> ins;
    for (auto const& v : l.at("inputs").as_array()) ins.push_back(value_ref_from(v));
    std::vector<TensorAttrs> outs;
    for (auto const& o : l.at("outputs").as_array()) {
      TensorAttrs t;
      t.shape = TensorShape::from_json(o.at("shape"));
      t.create_grad = o.at("create_grad").as_bool();
      if (o.contains("initializer")) t.initializer = o.at("initializer").dump();
      outs.push_back(t);
    }
    cg.g.add_node_with_id(static_cast<int>(l.at("id").as_int()),
                          LayerAttrs{normalize_attrs(OpAttrs::from_json(l.at("op"))), l.at("name").as_string()},
                          ins, outs);
  }
  return cg;
}

std::string ComputationGraph::as_dot() const {
  return digraph_as_dot(g.digraph(), [&](int id) {
    auto const& n = g.node(id);
    std::string s = n.label.name + "\n" + to_string(n.label.op.type);
    for (auto const& t : n.outputs) s += "\n" + t.shape.str();
    return s;
  });
}

// ===========================================================================
// ParallelComputationGraph
std::vector<OpAttrs> generate_weight_transform(const TensorShape& serial, const ParallelTensorShape& target) {
  if (serial != target.reduced_shape())
    throw FFError("generate_weight_transform: shape mismatch " + serial.str() + " vs " + target.str());
  std::vector<OpAttrs> ops;
  for (int d = 0; d < target.num_dims(); ++d)
    if (target.shard_dims[d].degree > 1) ops.push_back(make_repartition(d, target.shard_dims[d].degree));
  if (target.discard_copy_degree > 1) ops.push_back(make_replicate(target.discard_copy_degree));
  if (target.sum_degree > 1) {
    OpAttrs r = make_replicate(target.sum_degree);
    r.set("partial", true);
    ops.push_back(r);
  }
  return ops;
}

ValueRef ParallelComputationGraph::add_input(const ParallelTensorShape& shape, bool create_grad,
                                             const std::string& name) {
  OpAttrs a(OpType::INPUT);
  TensorShape s = shape.reduced_shape();
  a.set("dims", s.dims).set("data_type", to_string(s.dtype));
  a = normalize_attrs(a);
  int id = g.add_node(LayerAttrs{a, name}, {}, {ParallelTensorAttrs{shape, create_grad, ""}});
  return {id, 0};
}

ValueRef ParallelComputationGraph::add_weight(const TensorShape& serial, const ParallelTensorShape& target,
                                              const std::string& init, bool create_grad, const std::string& name) {
  OpAttrs a(OpType::WEIGHT);
  a.set("dims", serial.dims).set("data_type", to_string(serial.dtype)).set("initializer", init);
  a = normalize_attrs(a);
  int id = g.add_node(LayerAttrs{a, name}, {}, {ParallelTensorAttrs{lift_to_parallel(serial), create_grad, init}});
  ValueRef cur{id, 0};
  for (auto const& op : generate_weight_transform(serial, target)) cur = add_layer(op, {cur})[0];
  if (shape(cur) != target) throw FFError("add_weight: transform did not reach target " + target.str());
  return cur;
}

std::vector<ValueRef> ParallelComputationGraph::add_layer(const OpAttrs& op_in, const std::vector<ValueRef>& inputs,
                                                          const std::string& name) {
  OpAttrs op = normalize_attrs(op_in);
  int nd_in = num_data_inputs(op);
  int nw = num_weights(op);
  if (nd_in < 0) nd_in = static_cast<int>(inputs.size()) - nw;
  if (static_cast<int>(inputs.size()) != nd_in + nw)
    throw FFError(to_string(op.type) + ": expected " + std::to_string(nd_in + nw) + " incoming tensors");
  std::vector<ParallelTensorShape> din;
  for (int i = 0; i < nd_in; ++i) din.push_back(shape(inputs[i]));
  auto wexp = infer_parallel_weight_shapes(op, din);
  for (int i = 0; i < nw; ++i)
    if (shape(inputs[nd_in + i]) != wexp[i])
      throw FFError(to_string(op.type) + ": weight " + std::to_string(i) + " has parallel shape " +
                    shape(inputs[nd_in + i]).str() + ", expected " + wexp[i].str());
  auto outs = infer_parallel_output_shapes(op, din);
  std::vector<ParallelTensorAttrs> oa;
  bool grad = false;
  for (auto const& v : inputs) grad = grad || g.tensor(v).create_grad;
  for (auto const& s : outs) {
    bool fp = s.dtype == DataType::FLOAT || s.dtype == DataType::HALF || s.dtype == DataType::BFLOAT16 ||
              s.dtype == DataType::DOUBLE;
    oa.push_back(ParallelTensorAttrs{s, fp, ""});
  }
  int id = g.add_node(LayerAttrs{op, name}, inputs, oa);
  std::vector<ValueRef> r;
  for (size_t i = 0; i < outs.size(); ++i) r.push_back({id, static_cast<int>(i)});
  return r;
}

std::vector<ValueRef> ParallelComputationGraph::add_layer_auto_weights(const OpAttrs& op_in,
                                                                       const std::vector<ValueRef>& din,
                                                                       const std::string& name,
                                                                       const std::vector<std::string>& inits) {
  OpAttrs op = normalize_attrs(op_in);
  std::vector<ParallelTensorShape> ps;
  for (auto const& v : din) ps.push_back(shape(v));
  auto wshapes = infer_parallel_weight_shapes(op, ps);
  auto wnames = weight_names(op);
  std::vector<ValueRef> all = din;
  for (size_t i = 0; i < wshapes.size(); ++i) {
    std::string init = (i < inits.size() && !inits[i].empty()) ? inits[i] : default_initializer(op.type, wnames[i]);
    all.push_back(add_weight(wshapes[i].reduced_shape(), wshapes[i], init, true, name + "." + wnames[i]));
  }
  return add_layer(op, all, name);
}

ValueRef ParallelComputationGraph::parallel_partition(ValueRef x, int dim, int degree, const std::string& name) {
  return add_layer(make_repartition(dim, degree), {x}, name)[0];
}
ValueRef ParallelComputationGraph::parallel_combine(ValueRef x, int dim, int degree, const std::string& name) {
  return add_layer(make_combine(dim, degree), {x}, name)[0];
}
ValueRef ParallelComputationGraph::parallel_replicate(ValueRef x, int degree, const std::string& name) {
  return add_layer(make_replicate(degree), {x}, name)[0];
}
ValueRef ParallelComputationGraph::parallel_reduce(ValueRef x, int degree, const std::string& name) {
  return add_layer(make_reduction(degree), {x}, name)[0];
}

std::vector<ValueRef> ParallelComputationGraph::layer_weights(int node) const {
  auto const& n = g.node(node);
  if (n.label.op.type == OpType::INPUT || n.label.op.type == OpType::WEIGHT) return {};
  int nw = num_weights(n.label.op);
  return std::vector<ValueRef>(n.inputs.end() - nw, n.inputs.end());
}

std::vector<ValueRef> ParallelComputationGraph::layer_data_inputs(int node) const {
  auto const& n = g.node(node);
  if (n.label.op.type == OpType::INPUT || n.label.op.type == OpType::WEIGHT) return {};
  int nw = num_weights(n.label.op);
  return std::vector<ValueRef>(n.inputs.begin(), n.inputs.end() - nw);
}

bool ParallelComputationGraph::is_weight_path(int node) const {
  auto const& n = g.node(node);
  if (n.label.op.type == OpType::WEIGHT) return true;
  if (!is_parallel_op(n.label.op.type)) return false;
  return is_weight_path(n.inputs.at(0).node);
}

void ParallelComputationGraph::reinfer_shapes() {
  for (int id : g.topo_order()) {
    auto& n = g.node(id);
    auto t = n.label.op.type;
    if (t == OpType::INPUT || t == OpType::WEIGHT) continue;
    int nw = num_weights(n.label.op);
    std::vector<ParallelTensorShape> din;
    for (size_t i = 0; i + nw < n.inputs.size(); ++i) din.push_back(shape(n.inputs[i]));
    auto outs = infer_parallel_output_shapes(n.label.op, din);
    auto wexp = infer_parallel_weight_shapes(n.label.op, din);
    for (int i = 0; i < nw; ++i) {
      auto const& ws = shape(n.inputs[n.inputs.size() - nw + i]);
      if (ws != wexp[i])
        throw FFError("reinfer_shapes: " + n.label.name + " weight shape " + ws.str() + " != " + wexp[i].str());
    }
    if (outs.size() != n.outputs.size()) throw FFError("reinfer_shapes: output count changed");
    for (size_t i = 0; i < outs.size(); ++i) n.outputs[i].shape = outs[i];
  }
}

Json ParallelComputationGraph::to_json() const {
  Json j = Json::object();
  j["format"] = "ffmi355x.parallel_computation_graph.v1";
  Json layers = Json::array();
  for (int id : g.topo_order()) {
    auto const& n = g.node(id);
    Json l = Json::object();
    l["id"] = id;
    l["name"] = n.label.name;
    l["op"] = n.label.op.to_json();
    Json ins = Json::array();
    for (auto const& v : n.inputs) ins.push_back(value_ref_json(v));
    l["inputs"] = ins;
    Json outs = Json::array();
    for (auto const& t : n.outputs) {
      Json o = Json::object();
      o["shape"] = t.shape.to_json();
      o["create_grad"] = t.create_grad;
      if (!t.initializer.empty()) o["initializer"] = Json::parse(t.initializer);
      outs.push_back(o);
    }
    l["outputs"] = outs;
    layers.push_back(l);
  }
  j["layers"] = layers;
  return j;
}

ParallelComputationGraph ParallelComputationGraph::from_json(const Json& j) {
  ParallelComputationGraph p;
  for (auto const& l : j.at("layers").as_array()) {
    std::vector<ValueRef> ins;
    for (auto const& v : l.at("inputs").as_array()) ins.push_back(value_ref_from(v));
    std::vector<ParallelTensorAttrs> outs;
    for (auto const& o : l.at("outputs").as_array()) {
      ParallelTensorAttrs t;
      t.shape = ParallelTensorShape::from_json(o.at("shape"));
      t.create_grad = o.at("create_grad").as_bool();
      if (o.contains("initializer")) t.initializer = o.at("initializer").dump();
      outs.push_back(t);
    }
    p.g.add_node_with_id(static_cast<int>(l.at("id").as_int()),
                         LayerAttrs{normalize_attrs(OpAttrs::from_json(l.at("op"))), l.at("name").as_string()},
                         ins, outs);
  }
  return p;
}

std::string ParallelComputationGraph::as_dot() const {
  return digraph_as_dot(g.digraph(), [&](int id) {
    auto const& n = g.node(id);
    std::string s = (n.label.name.empty() ? "" : n.label.name + "\n") + n.label.op.str();
    for (auto const& t : n.outputs) s += "\n" + t.shape.str();
    return s;
  });
}

size_t ParallelComputationGraph::structural_hash() const {
  std::vector<size_t> h(g.next_id(), 0);
  std::vector<size_t> all;
  all.reserve(g.num_nodes());
  for (int id : g.topo_order()) {
    auto const& n = g.node(id);
    size_t x = n.label.op.hash();
    for (auto const& v : n.inputs) x = hash_combine(x, hash_combine(h[v.node], static_cast<size_t>(v.idx)));
    for (auto const& t : n.outputs) x = hash_combine(x, std::hash<ParallelTensorShape>()(t.shape));
    h[id] = x;
    all.push_back(x);
  }
  std::sort(all.begin(), all.end());
  size_t r = 0x1234;
  for (auto x : all) r = hash_combine(r, x);
  return r;
}

bool ParallelComputationGraph::structurally_equal(const ParallelComputationGraph& o) const {
  if (g.num_nodes() != o.g.num_nodes()) return false;
  return structural_hash() == o.structural_hash();
}

int ParallelComputationGraph::num_operator_nodes() const {
  int c = 0;
  for (int id : g.node_ids()) {
    auto t = g.node(id).label.op.type;
    if (t != OpType::INPUT && t != OpType::WEIGHT && !is_weight_path(id)) ++c;
  }
  return c;
}

ParallelComputationGraph pcg_from_computation_graph(const ComputationGraph& cg, std::map<int, int>* mapping) {
  ParallelComputationGraph p;
  std::map<int, int> m;
  for (int id : cg.g.topo_order()) {
    auto const& n = cg.g.node(id);
    auto t = n.label.op.type;
    int nid;
    if (t == OpType::INPUT) {
      nid = p.add_input(lift_to_parallel(n.outputs[0].shape), n.outputs[0].create_grad, n.label.name).node;
    } else if (t == OpType::WEIGHT) {
      nid = p.add_weight(n.outputs[0].shape, lift_to_parallel(n.outputs[0].shape), n.outputs[0].initializer,
                         n.outputs[0].create_grad, n.label.name)
                .node;
    } else {
      std::vector<ValueRef> ins;
      for (auto const& v : n.inputs) ins.push_back({m.at(v.node), v.idx});
      nid = p.add_layer(n.label.op, ins, n.label.name)[0].node;
    }
    m[id] = nid;
  }
  if (mapping) *mapping = m;
  return p;
}

ParallelComputationGraph data_parallel_pcg(const ComputationGraph& cg, int degree) {
  ParallelComputationGraph p;
  std::map<ValueRef, ValueRef> vm;  // cg value -> pcg value
  // Bring a tensor to fully-unpartitioned (degree-1) form.
  auto gather_all = [&](ValueRef v) {
    auto s = p.shape(v);
    if (s.sum_degree > 1) v = p.parallel_reduce(v, s.sum_degree);
    s = p.shape(v);
    for (int d = 0; d < s.num_dims(); ++d)
      if (s.shard_dims[d].degree > 1) v = p.parallel_combine(v, d, s.shard_dims[d].degree);
    return v;
  };
  for (int id : cg.g.topo_order()) {
    auto const& n = cg.g.node(id);
    auto t = n.label.op.type;
    if (t == OpType::WEIGHT) continue;  // created on demand with the right degrees
    if (t == OpType::INPUT) {
      auto const& s = n.outputs[0].shape;
      ValueRef v = p.add_input(lift_to_parallel(s), n.outputs[0].create_grad, n.label.name);
      const bool replicated = n.label.op.has("replicated") && n.label.op.b("replicated");
      if (degree > 1 && !replicated && s.num_dims() > 0 && s.dims[0] % degree == 0)
        v = p.parallel_partition(v, 0, degree);
      vm[{id, 0}] = v;
      continue;
    }
    auto data = cg.layer_data_inputs(id);
    auto wts = cg.layer_weights(id);
    std::vector<ValueRef> din;
    for (auto const& v : data) din.push_back(vm.at(v));
    std::vector<ParallelTensorShape> ps;
    for (auto const& v : din) ps.push_back(p.shape(v));
    if (!is_valid_parallelization(n.label.op, ps)) {
      for (auto& v : din) v = gather_all(v);
      ps.clear();
      for (auto const& v : din) ps.push_back(p.shape(v));
    }
    auto wshapes = infer_parallel_weight_shapes(n.label.op, ps);
    std::vector<ValueRef> all = din;
    for (size_t i = 0; i < wts.size(); ++i) {
      auto const& wn = cg.g.node(wts[i].node);
      all.push_back(p.add_weight(wn.outputs[0].shape, wshapes[i], wn.outputs[0].initializer,
                                 wn.outputs[0].create_grad, wn.label.name));
    }
    auto outs = p.add_layer(n.label.op, all, n.label.name);
    for (size_t i = 0; i < outs.size(); ++i) {
      ValueRef o = outs[i];
      auto s = p.shape(o);
      // resolve pending sums and re-shard on the sample dim for the next op
      if (s.sum_degree > 1) {
        o = p.parallel_reduce(o, s.sum_degree);
        s = p.shape(o);
      }
      if (degree > 1 && s.total_parallel_degree() == 1 && s.num_dims() > 0 && s.shard_dims[0].size % degree == 0)
        o = p.parallel_partition(o, 0, degree);
      vm[{id, static_cast<int>(i)}] = o;
    }
  }
  return p;
}

}  // namespace ff
