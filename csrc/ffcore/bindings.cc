// pybind11 bindings for the ffcore C++ library (module `_ffcore`).
//
// Parity: replaces the reference's C FFI headers (lib/*/ffi/include/flexflow/*.h)
// and the cffi sketch in bindings/python; IR objects cross the boundary either
// as bound classes or as JSON strings (the file format v1).
#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "ff/computation_graph.h"
#include "ff/graph.h"
#include "ff/json.h"
#include "ff/op_attrs.h"
#include "ff/sp.h"
#include "ff/types.h"
#include "bindings_ext.h"

namespace py = pybind11;
using namespace ff;

namespace ff {
AttrValue py_to_attr(const py::handle& o) {
  if (py::isinstance<py::bool_>(o)) return o.cast<bool>();
  if (py::isinstance<py::int_>(o)) return o.cast<int64_t>();
  if (py::isinstance<py::float_>(o)) return o.cast<double>();
  if (py::isinstance<py::str>(o)) return o.cast<std::string>();
  if (py::isinstance<py::list>(o) || py::isinstance<py::tuple>(o)) {
    std::vector<int64_t> v;
    for (auto x : o) v.push_back(x.cast<int64_t>());
    return v;
  }
  // enums / numpy scalars
  if (py::hasattr(o, "__index__")) return o.attr("__index__")().cast<int64_t>();
  throw FFError("unsupported attribute value type");
}

py::object attr_to_py(const AttrValue& v) {
  switch (v.index()) {
    case 0: return py::int_(std::get<int64_t>(v));
    case 1: return py::float_(std::get<double>(v));
    case 2: return py::bool_(std::get<bool>(v));
    case 3: return py::str(std::get<std::string>(v));
    default: return py::cast(std::get<std::vector<int64_t>>(v));
  }
}

OpAttrs make_op(const std::string& type, const py::dict& kw) {
  OpAttrs a(optype_from_string(type));
  for (auto item : kw) a.attrs[item.first.cast<std::string>()] = py_to_attr(item.second);
  return normalize_attrs(a);
}
}  // namespace ff

PYBIND11_MODULE(_ffcore, m) {
  m.doc() = "flexflow_train_amd native core: IR, shape inference, PCG, search";

  py::register_exception<FFError>(m, "FFError", PyExc_ValueError);

  py::enum_<DataType>(m, "DataType")
      .value("BOOL", DataType::BOOL)
      .value("INT32", DataType::INT32)
      .value("INT64", DataType::INT64)
      .value("HALF", DataType::HALF)
      .value("BFLOAT16", DataType::BFLOAT16)
      .value("FLOAT", DataType::FLOAT)
      .value("DOUBLE", DataType::DOUBLE)
      .value("FP8_E4M3", DataType::FP8_E4M3)
      .value("NONE", DataType::NONE);
  m.def("datatype_from_string", &datatype_from_string);
  m.def("datatype_to_string", [](DataType d) { return to_string(d); });
  m.def("size_of", &size_of);

  {
    auto e = py::enum_<OpType>(m, "OpType");
    for (auto t : all_op_types()) e.value(to_string(t).c_str(), t);
  }
  m.def("optype_from_string", &optype_from_string);
  m.def("optype_to_string", [](OpType t) { return to_string(t); });
  m.def("is_parallel_op", &is_parallel_op);

  py::class_<TensorShape>(m, "TensorShape")
      .def(py::init([](std::vector<int64_t> dims, DataType dt) { return TensorShape{std::move(dims), dt}; }),
           py::arg("dims"), py::arg("dtype") = DataType::FLOAT)
      .def_readwrite("dims", &TensorShape::dims)
      .def_readwrite("dtype", &TensorShape::dtype)
      .def("num_elements", &TensorShape::num_elements)
      .def("size_bytes", &TensorShape::size_bytes)
      .def("to_json", [](const TensorShape& s) { return s.to_json().dump(); })
      .def_static("from_json", [](const std::string& s) { return TensorShape::from_json(Json::parse(s)); })
      .def("__eq__", &TensorShape::operator==)
      .def("__hash__", [](const TensorShape& s) { return std::hash<TensorShape>()(s); })
      .def("__repr__", &TensorShape::str);

  py::class_<ShardParallelDim>(m, "ShardParallelDim")
      .def(py::init([](int64_t size, int degree) { return ShardParallelDim{size, degree}; }))
      .def_readwrite("size", &ShardParallelDim::size)
      .def_readwrite("degree", &ShardParallelDim::degree)
      .def("__eq__", &ShardParallelDim::operator==)
      .def("__repr__", [](const ShardParallelDim& d) {
        return std::to_string(d.size) + "/" + std::to_string(d.degree);
      });

  py::class_<ParallelTensorShape>(m, "ParallelTensorShape")
      .def(py::init([](std::vector<int64_t> dims, std::vector<int> degrees, int sum, int copy, DataType dt) {
             TensorShape s{std::move(dims), dt};
             if (degrees.empty()) degrees.assign(s.dims.size(), 1);
             return lift_to_parallel_with_degrees(s, sum, copy, degrees);
           }),
           py::arg("dims"), py::arg("degrees") = std::vector<int>{}, py::arg("sum_degree") = 1,
           py::arg("discard_copy_degree") = 1, py::arg("dtype") = DataType::FLOAT)
      .def_readwrite("shard_dims", &ParallelTensorShape::shard_dims)
      .def_readwrite("sum_degree", &ParallelTensorShape::sum_degree)
      .def_readwrite("discard_copy_degree", &ParallelTensorShape::discard_copy_degree)
      .def_readwrite("dtype", &ParallelTensorShape::dtype)
      .def("shard_degrees", &ParallelTensorShape::shard_degrees)
      .def("total_parallel_degree", &ParallelTensorShape::total_parallel_degree)
      .def("reduced_shape", &ParallelTensorShape::reduced_shape)
      .def("piece_shape", &ParallelTensorShape::piece_shape)
      .def("is_valid", &ParallelTensorShape::is_valid)
      .def("to_json", [](const ParallelTensorShape& s) { return s.to_json().dump(); })
      .def_static("from_json", [](const std::string& s) { return ParallelTensorShape::from_json(Json::parse(s)); })
      .def("__eq__", &ParallelTensorShape::operator==)
      .def("__hash__", [](const ParallelTensorShape& s) { return std::hash<ParallelTensorShape>()(s); })
      .def("__repr__", &ParallelTensorShape::str);
  m.def("lift_to_parallel", &lift_to_parallel);

  py::class_<OpAttrs>(m, "OpAttrs")
      .def(py::init([](const std::string& type, py::kwargs kw) { return make_op(type, kw); }))
      .def_readonly("type", &OpAttrs::type)
      .def_property_readonly("op_type", [](const OpAttrs& a) { return to_string(a.type); })
      .def("get", [](const OpAttrs& a, const std::string& k) {
        auto it = a.attrs.find(k);
        if (it == a.attrs.end()) throw py::key_error(k);
        return attr_to_py(it->second);
      })
      .def("has", &OpAttrs::has)
      .def("items", [](const OpAttrs& a) {
        py::dict d;
        for (auto const& kv : a.attrs) d[py::str(kv.first)] = attr_to_py(kv.second);
        return d;
      })
      .def("to_json", [](const OpAttrs& a) { return a.to_json().dump(); })
      .def_static("from_json", [](const std::string& s) { return normalize_attrs(OpAttrs::from_json(Json::parse(s))); })
      .def("__eq__", &OpAttrs::operator==)
      .def("__hash__", &OpAttrs::hash)
      .def("__repr__", &OpAttrs::str);

  m.def("infer_output_shapes", &infer_output_shapes);
  m.def("infer_weight_shapes", &infer_weight_shapes);
  m.def("infer_parallel_output_shapes", &infer_parallel_output_shapes);
  m.def("infer_parallel_weight_shapes", &infer_parallel_weight_shapes);
  m.def("is_valid_parallelization", &is_valid_parallelization);
  m.def("num_weights", &num_weights);
  m.def("weight_names", &weight_names);
  m.def("num_data_inputs", &num_data_inputs);
  m.def("estimate_op_work", [](const OpAttrs& a, const std::vector<TensorShape>& i,
                               const std::vector<TensorShape>& w, const std::vector<TensorShape>& o) {
    auto r = estimate_op_work(a, i, w, o);
    return py::dict(py::arg("flops") = r.flops, py::arg("bytes") = r.bytes,
                    py::arg("matmul_like") = r.matmul_like);
  });
  m.def("default_initializer", &default_initializer);
  m.def("generate_weight_transform", &generate_weight_transform);

  py::class_<ValueRef>(m, "ValueRef")
      .def(py::init([](int n, int i) { return ValueRef{n, i}; }), py::arg("node"), py::arg("idx") = 0)
      .def_readonly("node", &ValueRef::node)
      .def_readonly("idx", &ValueRef::idx)
      .def("__eq__", &ValueRef::operator==)
      .def("__hash__", [](const ValueRef& v) { return std::hash<int64_t>()((int64_t(v.node) << 8) ^ v.idx); })
      .def("__repr__", [](const ValueRef& v) {
        return "ValueRef(" + std::to_string(v.node) + ", " + std::to_string(v.idx) + ")";
      });

  py::class_<ComputationGraph>(m, "ComputationGraph")
      .def(py::init<>())
      .def("set_input_replicated", &ComputationGraph::set_input_replicated, py::arg("node"))
      .def("create_input", &ComputationGraph::create_input, py::arg("shape"), py::arg("create_grad") = true,
           py::arg("name") = "")
      .def("create_weight", &ComputationGraph::create_weight, py::arg("shape"), py::arg("initializer"),
           py::arg("create_grad") = true, py::arg("name") = "")
      .def("add_layer", &ComputationGraph::add_layer, py::arg("op"), py::arg("inputs"), py::arg("name") = "",
           py::arg("weight_initializers") = std::vector<std::string>{})
      .def("add_layer_with_weights", &ComputationGraph::add_layer_with_weights)
      .def("shape", &ComputationGraph::shape)
      .def("topo_order", &ComputationGraph::layers_in_topo_order)
      .def("layer_weights", &ComputationGraph::layer_weights)
      .def("layer_data_inputs", &ComputationGraph::layer_data_inputs)
      .def("find_layer", &ComputationGraph::find_layer)
      .def("num_layers", [](const ComputationGraph& c) { return c.g.num_nodes(); })
      .def("layer_op", [](const ComputationGraph& c, int n) { return c.g.node(n).label.op; })
      .def("layer_name", [](const ComputationGraph& c, int n) { return c.g.node(n).label.name; })
      .def("layer_inputs", [](const ComputationGraph& c, int n) { return c.g.node(n).inputs; })
      .def("num_outputs", [](const ComputationGraph& c, int n) { return c.g.node(n).outputs.size(); })
      .def("create_grad", [](const ComputationGraph& c, ValueRef v) { return c.g.tensor(v).create_grad; })
      .def("initializer", [](const ComputationGraph& c, ValueRef v) { return c.g.tensor(v).initializer; })
      .def("uses", [](const ComputationGraph& c, ValueRef v) { return c.g.uses(v); })
      .def("to_json", [](const ComputationGraph& c) { return c.to_json().dump(); })
      .def_static("from_json", [](const std::string& s) { return ComputationGraph::from_json(Json::parse(s)); })
      .def("as_dot", &ComputationGraph::as_dot);

  py::class_<ParallelComputationGraph>(m, "ParallelComputationGraph")
      .def(py::init<>())
      .def("add_input", &ParallelComputationGraph::add_input, py::arg("shape"), py::arg("create_grad") = true,
           py::arg("name") = "")
      .def("add_weight", &ParallelComputationGraph::add_weight, py::arg("serial_shape"), py::arg("target"),
           py::arg("initializer"), py::arg("create_grad") = true, py::arg("name") = "")
      .def("add_layer", &ParallelComputationGraph::add_layer, py::arg("op"), py::arg("inputs"),
           py::arg("name") = "")
      .def("add_layer_auto_weights", &ParallelComputationGraph::add_layer_auto_weights, py::arg("op"),
           py::arg("inputs"), py::arg("name") = "",
           py::arg("weight_initializers") = std::vector<std::string>{})
      .def("parallel_partition", &ParallelComputationGraph::parallel_partition, py::arg("x"), py::arg("dim"),
           py::arg("degree"), py::arg("name") = "")
      .def("parallel_combine", &ParallelComputationGraph::parallel_combine, py::arg("x"), py::arg("dim"),
           py::arg("degree"), py::arg("name") = "")
      .def("parallel_replicate", &ParallelComputationGraph::parallel_replicate, py::arg("x"),
           py::arg("degree"), py::arg("name") = "")
      .def("parallel_reduce", &ParallelComputationGraph::parallel_reduce, py::arg("x"), py::arg("degree"),
           py::arg("name") = "")
      .def("shape", &ParallelComputationGraph::shape)
      .def("topo_order", [](const ParallelComputationGraph& p) { return p.g.topo_order(); })
      .def("layer_weights", &ParallelComputationGraph::layer_weights)
      .def("layer_data_inputs", &ParallelComputationGraph::layer_data_inputs)
      .def("is_weight_path", &ParallelComputationGraph::is_weight_path)
      .def("num_layers", [](const ParallelComputationGraph& p) { return p.g.num_nodes(); })
      .def("num_operator_nodes", &ParallelComputationGraph::num_operator_nodes)
      .def("layer_op", [](const ParallelComputationGraph& p, int n) { return p.g.node(n).label.op; })
      .def("layer_name", [](const ParallelComputationGraph& p, int n) { return p.g.node(n).label.name; })
      .def("layer_inputs", [](const ParallelComputationGraph& p, int n) { return p.g.node(n).inputs; })
      .def("num_outputs", [](const ParallelComputationGraph& p, int n) { return p.g.node(n).outputs.size(); })
      .def("create_grad", [](const ParallelComputationGraph& p, ValueRef v) { return p.g.tensor(v).create_grad; })
      .def("initializer", [](const ParallelComputationGraph& p, ValueRef v) { return p.g.tensor(v).initializer; })
      .def("uses", [](const ParallelComputationGraph& p, ValueRef v) { return p.g.uses(v); })
      .def("reinfer_shapes", &ParallelComputationGraph::reinfer_shapes)
      .def("structural_hash", &ParallelComputationGraph::structural_hash)
      .def("structurally_equal", &ParallelComputationGraph::structurally_equal)
      .def("to_json", [](const ParallelComputationGraph& p) { return p.to_json().dump(); })
      .def_static("from_json",
                  [](const std::string& s) { return ParallelComputationGraph::from_json(Json::parse(s)); })
      .def("as_dot", &ParallelComputationGraph::as_dot);

  m.def("pcg_from_computation_graph", [](const ComputationGraph& cg) {
    std::map<int, int> mp;
    auto p = pcg_from_computation_graph(cg, &mp);
    return py::make_tuple(p, mp);
  });
  m.def("data_parallel_pcg", &data_parallel_pcg);

  m.def("json_roundtrip", [](const std::string& s) { return Json::parse(s).dump(); });

  // ---- graph library (lib/utils/graph parity), DiGraph given as (nodes, edges)
  auto mkg = [](const std::vector<int>& nodes, const std::vector<std::pair<int, int>>& edges) {
    DiGraph g;
    for (int n : nodes) g.add_node(n);
    for (auto const& e : edges) g.add_edge(e.first, e.second);
    return g;
  };
  auto edges_of = [](const DiGraph& g) {
    std::vector<std::pair<int, int>> r;
    for (auto const& kv : g.succ)
      for (int s : kv.second) r.emplace_back(kv.first, s);
    return r;
  };
  auto g = m.def_submodule("graph", "DiGraph algorithms over (nodes, edges)");
  g.def("topological_order", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return topological_order(mkg(n, e));
  });
  g.def("is_acyclic", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) { return is_acyclic(mkg(n, e)); });
  g.def("transitive_closure", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return edges_of([&] {
      DiGraph r;
      for (auto const& kv : transitive_closure(mkg(n, e))) {
        r.add_node(kv.first);
        for (int s : kv.second) r.add_edge(kv.first, s);
      }
      return r;
    }());
  });
  g.def("transitive_reduction", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return edges_of(transitive_reduction(mkg(n, e)));
  });
  g.def("dominators", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) { return dominators(mkg(n, e)); });
  g.def("post_dominators",
        [=](std::vector<int> n, std::vector<std::pair<int, int>> e) { return post_dominators(mkg(n, e)); });
  g.def("immediate_dominators",
        [=](std::vector<int> n, std::vector<std::pair<int, int>> e) { return immediate_dominators(mkg(n, e)); });
  g.def("immediate_post_dominators", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return immediate_post_dominators(mkg(n, e));
  });
  g.def("weakly_connected_components", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return weakly_connected_components(mkg(n, e));
  });
  g.def("longest_path", [=](std::vector<int> n, std::vector<std::pair<int, int>> e, std::map<int, double> w) {
    return longest_path(mkg(n, e), [&](int x) { auto it = w.find(x); return it == w.end() ? 1.0 : it->second; });
  });
  g.def("find_isomorphism", [=](std::vector<int> na, std::vector<std::pair<int, int>> ea, std::vector<int> nb,
                                std::vector<std::pair<int, int>> eb, std::map<int, std::string> la,
                                std::map<int, std::string> lb) -> py::object {
    auto A = mkg(na, ea), B = mkg(nb, eb);
    auto r = find_isomorphism(A, B, [&](int x) { auto it = la.find(x); return it == la.end() ? std::string() : it->second; },
                              [&](int x) { auto it = lb.find(x); return it == lb.end() ? std::string() : it->second; });
    if (!r) return py::none();
    return py::cast(*r);
  }, py::arg("nodes_a"), py::arg("edges_a"), py::arg("nodes_b"), py::arg("edges_b"),
     py::arg("labels_a") = std::map<int, std::string>{}, py::arg("labels_b") = std::map<int, std::string>{});
  g.def("inverse_line_graph", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) -> py::object {
    auto r = inverse_line_graph(mkg(n, e));
    if (!r) return py::none();
    return py::make_tuple(std::vector<int>(r->h.nodes.begin(), r->h.nodes.end()), edges_of(r->h), r->edge);
  });
  g.def("as_dot", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) {
    return digraph_as_dot(mkg(n, e), [](int x) { return std::to_string(x); });
  });
  // SP tree utilities on the decomposition of a DiGraph
  auto sp_of = [=](const std::vector<int>& n, const std::vector<std::pair<int, int>>& e) {
    return get_relaxed_sp_decomposition(mkg(n, e));
  };
  g.def("sp_paths_to_leaf", [=](std::vector<int> n, std::vector<std::pair<int, int>> e, int node) {
    return find_paths_to_leaf(sp_of(n, e), node);
  });
  g.def("sp_subtree_leaves_at_path", [=](std::vector<int> n, std::vector<std::pair<int, int>> e,
                                         std::vector<int> path) -> py::object {
    auto t = sp_of(n, e);
    const int i = get_subtree_at_path(t, path);
    if (i < 0) return py::none();
    return py::cast(t.leaves(i));
  });
  // strict SP decomposition as binary nested tuples (None if not SP)
  g.def("sp_decomposition", [=](std::vector<int> n, std::vector<std::pair<int, int>> e) -> py::object {
    auto t = get_series_parallel_decomposition(mkg(n, e));
    if (!t || t->root < 0) return py::none();
    std::function<py::object(int)> conv = [&](int i) -> py::object {
      const auto& x = t->e[i];
      if (x.kind == SPTree::LEAF) return py::int_(x.node);
      return py::make_tuple(x.kind == SPTree::SERIES ? "S" : "P", conv(x.left), conv(x.right));
    };
    return conv(t->root);
  });
  g.def("sp_associative", [=](std::vector<int> n, std::vector<std::pair<int, int>> e, bool left) {
    auto t = sp_of(n, e);
    auto r = left ? left_associative(t) : right_associative(t);
    // binary nested tuples: leaf = node id, split = ("S"|"P", left, right)
    std::function<py::object(int)> conv = [&](int i) -> py::object {
      const auto& x = r.e[i];
      if (x.kind == SPTree::LEAF) return py::int_(x.node);
      return py::make_tuple(x.kind == SPTree::SERIES ? "S" : "P", conv(x.left), conv(x.right));
    };
    return r.root < 0 ? py::object(py::none()) : conv(r.root);
  });

  register_ext_bindings(m);
  register_data_bindings(m);
}
