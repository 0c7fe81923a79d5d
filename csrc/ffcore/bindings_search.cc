// Bindings for the machine model, cost model, SP decomposition, lowering,
// simulator, machine mapping, substitutions and strategy search.
// Structured results cross the boundary as JSON strings (parsed by
// flexflow_train_amd.search.native); graphs stay native objects.
#include <limits>

#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bindings_ext.h"
#include "ff/mapping.h"
#include "ff/memory_plan.h"
#include "ff/network.h"
#include "ff/models.h"
#include "ff/parallelize.h"
#include "ff/search.h"
#include "ff/simulator.h"
#include "ff/sp.h"
#include "ff/substitution.h"

namespace py = pybind11;

namespace ff {

namespace {

std::map<int, std::vector<int>> views_to_py(const std::map<int, Placement>& v) {
  return std::map<int, std::vector<int>>(v.begin(), v.end());
}

// ---- the generic machine-mapping DP over a JSON-described problem with a
// table cost estimator (the reference's make_fake_cost_estimator cases,
// lib/compiler/test/src/compiler/machine_mapping/get_optimal_machine_mapping.cc)
BinaryTreePath path_from(const std::string& s) {
  BinaryTreePath p;
  for (char c : s)
    if (c == 'L' || c == 'R') p.push_back(c == 'R');
  return p;
}
std::string path_to(const BinaryTreePath& p) {
  std::string s;
  for (int x : p) s += x ? 'R' : 'L';
  return s;
}

int tree_from_json(MMProblemTree& t, const Json& j) {
  if (j.contains("leaf")) {
    UnmappedOpKey k;
    k.id = j.at("leaf").as_string();
    if (j.contains("task_space")) {
      std::vector<int64_t> ts;
      for (auto const& x : j.at("task_space").as_array()) ts.push_back(x.as_int());
      ParallelTensorShape o;
      for (size_t i = 0; i + 2 < ts.size(); ++i) o.shard_dims.push_back({ts[i], static_cast<int>(ts[i])});
      o.sum_degree = ts.size() >= 2 ? static_cast<int>(ts[ts.size() - 2]) : 1;
      o.discard_copy_degree = ts.empty() ? 1 : static_cast<int>(ts.back());
      k.outputs.push_back(o);
    }
    return t.add_leaf(k);
  }
  int l = tree_from_json(t, j.at("left"));
  int r = tree_from_json(t, j.at("right"));
  if (j.at("kind").as_string() == "parallel") return t.add_parallel(l, r);
  std::vector<AbstractedSingleTensorMovement> mv;
  if (j.contains("movement"))
    for (auto const& m : j.at("movement").as_array()) {
      AbstractedSingleTensorMovement a;
      for (auto const& x : m.at("src").as_array()) a.src.insert(path_from(x.as_string()));
      for (auto const& x : m.at("dst").as_array()) a.dst.insert(path_from(x.as_string()));
      mv.push_back(a);
    }
  return t.add_series(mv, l, r);
}

struct TableEstimator : MMCostEstimator {
  std::map<std::string, double> ops, moves;
  double default_op = std::numeric_limits<double>::infinity();
  double default_move = std::numeric_limits<double>::infinity();
  double estimate_op(const UnmappedOpKey& k, const MachineView& v) const override {
    auto it = ops.find(k.id + "@" + v.str());
    return it == ops.end() ? default_op : it->second;
  }
  static std::string move_key(const std::vector<SingleTensorMovement>& m) {
    std::string s;
    for (auto const& x : m) {
      s += "[";
      for (auto const& v : x.src) s += v.str() + ",";
      s += "->";
      for (auto const& v : x.dst) s += v.str() + ",";
      s += "]";
    }
    return s;
  }
  double estimate_movement(const std::vector<SingleTensorMovement>& m) const override {
    auto it = moves.find(move_key(m));
    return it == moves.end() ? default_move : it->second;
  }
};

MachineResource resource_from(const Json& j) {
  MachineResource r;
  if (j.contains("node_offset")) r.node_offset = static_cast<int>(j.at("node_offset").as_int());
  if (j.contains("gpu_offset")) r.gpu_offset = static_cast<int>(j.at("gpu_offset").as_int());
  r.num_nodes = static_cast<int>(j.at("num_nodes").as_int());
  r.gpus_per_node = static_cast<int>(j.at("gpus_per_node").as_int());
  return r;
}

}  // namespace

void register_ext_bindings(py::module_& m) {
  // ---- machine
  py::class_<MachineSpecification>(m, "MachineSpecification")
      .def(py::init<>())
      .def_static("mi355x", &MachineSpecification::mi355x, py::arg("num_nodes") = 1, py::arg("gpus_per_node") = 8)
      .def_readwrite("num_nodes", &MachineSpecification::num_nodes)
      .def_readwrite("num_cpus_per_node", &MachineSpecification::num_cpus_per_node)
      .def_readwrite("num_gpus_per_node", &MachineSpecification::num_gpus_per_node)
      .def_readwrite("inter_node_bandwidth", &MachineSpecification::inter_node_bandwidth)
      .def_readwrite("intra_node_bandwidth", &MachineSpecification::intra_node_bandwidth)
      .def_readwrite("peak_bf16_flops", &MachineSpecification::peak_bf16_flops)
      .def_readwrite("peak_fp32_flops", &MachineSpecification::peak_fp32_flops)
      .def_readwrite("mfma_efficiency", &MachineSpecification::mfma_efficiency)
      .def_readwrite("hbm_bandwidth", &MachineSpecification::hbm_bandwidth)
      .def_readwrite("hbm_capacity", &MachineSpecification::hbm_capacity)
      .def_readwrite("kernel_launch_overhead", &MachineSpecification::kernel_launch_overhead)
      .def_readwrite("collective_latency", &MachineSpecification::collective_latency)
      .def_readwrite("xgmi_links", &MachineSpecification::xgmi_links)
      .def_readwrite("xgmi_link_bandwidth", &MachineSpecification::xgmi_link_bandwidth)
      .def_readwrite("collective_bw", &MachineSpecification::collective_bw)
      .def_readwrite("all_to_all_bw", &MachineSpecification::all_to_all_bw)
      .def("num_devices", &MachineSpecification::num_devices)
      .def("to_json", [](const MachineSpecification& s) { return s.to_json().dump(); })
      .def_static("from_json", [](const std::string& s) { return MachineSpecification::from_json(Json::parse(s)); });

  py::class_<NetworkTopology>(m, "NetworkTopology")
      .def_readonly("num_devices", &NetworkTopology::num_devices)
      .def_readonly("num_vertices", &NetworkTopology::num_vertices)
      .def_readonly("name", &NetworkTopology::name)
      .def("num_links", [](const NetworkTopology& t) { return t.links.size(); })
      .def_static("fully_connected", &NetworkTopology::fully_connected)
      .def_static("big_switch", &NetworkTopology::big_switch)
      .def_static("flat_deg_constraint", &NetworkTopology::flat_deg_constraint)
      .def_static("mi355x_cluster", &NetworkTopology::mi355x_cluster, py::arg("nodes"), py::arg("gpus_per_node") = 8,
                  py::arg("xgmi_bw") = 64e9, py::arg("xgmi_lat") = 1e-6, py::arg("nic_bw") = 50e9,
                  py::arg("nic_lat") = 5e-6)
      .def_static("from_config_text", [](const std::string& t) {
        MachineSpecification spec;
        auto topo = NetworkTopology::from_config_text(t, &spec);
        return py::make_tuple(topo, spec);
      })
      .def_static("from_config_file", [](const std::string& p) {
        MachineSpecification spec;
        auto topo = NetworkTopology::from_config_file(p, &spec);
        return py::make_tuple(topo, spec);
      })
      .def("to_json", [](const NetworkTopology& t) { return t.to_json().dump(); });
  py::class_<NetworkModel>(m, "NetworkModel")
      .def(py::init([](const NetworkTopology& t, const std::string& routing, int max_rings) {
             return NetworkModel(t, routing == "weighted" ? RoutingStrategy::WEIGHTED_SHORTEST_PATH
                                                          : RoutingStrategy::SHORTEST_PATH_ECMP, max_rings);
           }),
           py::arg("topology"), py::arg("routing") = "ecmp", py::arg("max_rings") = 4)
      .def("routes", &NetworkModel::routes)
      .def("p2p_time", &NetworkModel::p2p_time)
      .def("all_reduce_time", &NetworkModel::all_reduce_time)
      .def("all_gather_time", &NetworkModel::all_gather_time)
      .def("all_to_all_time", &NetworkModel::all_to_all_time)
      .def("calibrate", [](const NetworkModel& nm, MachineSpecification spec, double probe) {
        nm.calibrate(spec, probe);
        return spec;
      }, py::arg("spec"), py::arg("probe_bytes") = 256.0 * (1 << 20));

  m.def("operator_task_space", &operator_task_space);
  m.def("get_allowed_machine_views", [](const std::vector<int>& ts, const MachineSpecification& spec) {
    std::vector<std::string> r;
    for (auto const& v : get_allowed_machine_views(ts, spec)) r.push_back(v.to_json().dump());
    return r;
  });
  m.def("get_machine_space_coordinate",
        [](const std::vector<int>& ts, const std::string& view, const std::vector<int>& coord,
           const MachineSpecification& spec) -> py::object {
          auto c = get_machine_space_coordinate(ts, MachineView::from_json(Json::parse(view)), coord, spec);
          if (!c) return py::none();
          return py::make_tuple(c->node_idx, c->device_idx);
        });
  // start-invariant views as JSON {"dimensions": [...]} (the MachineView
  // encoding without "start")
  m.def("start_invariant_from_machine_view", [](const std::string& view) {
    Json j = MachineView::from_json(Json::parse(view)).to_json();
    Json o = Json::object();
    o["dimensions"] = j.at("dimensions");
    return o.dump();
  });
  m.def("machine_view_from_start_invariant", [](const std::string& simv, int node, int device) {
    Json j = Json::parse(simv);
    j["start"] = Json(std::vector<int64_t>{node, device});
    return MachineView::from_json(j).to_json().dump();
  });
  m.def("get_machine_space_offset",
        [](const std::vector<int>& ts, const std::string& simv, const std::vector<int>& coord,
           const MachineSpecification& spec) -> py::object {
          Json j = Json::parse(simv);
          j["start"] = Json(std::vector<int64_t>{0, 0});
          auto c = get_machine_space_offset(ts, start_invariant_from_machine_view(MachineView::from_json(j)), coord,
                                            spec);
          if (!c) return py::none();
          return py::make_tuple(c->node_idx, c->device_idx);
        });
  m.def("get_device_ids", [](const std::vector<int>& ts, const std::string& view, const MachineSpecification& spec) {
    return get_device_ids(ts, MachineView::from_json(Json::parse(view)), spec);
  });
  m.def("block_machine_view", [](const std::vector<int>& ts, int start, int size, const MachineSpecification& spec) {
    return block_machine_view(ts, DeviceBlock{start, size}, spec).to_json().dump();
  });
  m.def("get_resource_splits", [](int start, int size) {
    std::vector<std::pair<std::pair<int, int>, std::pair<int, int>>> r;
    for (auto const& s : get_resource_splits(DeviceBlock{start, size}))
      r.push_back({{s.first.start, s.first.size}, {s.second.start, s.second.size}});
    return r;
  });
  m.def("collective_cost", [](const std::string& kind, double bytes, int p, const MachineSpecification& s) {
    if (kind == "all_reduce") return CollectiveCost::all_reduce(bytes, p, s);
    if (kind == "all_gather") return CollectiveCost::all_gather(bytes, p, s);
    if (kind == "reduce_scatter") return CollectiveCost::reduce_scatter(bytes, p, s);
    if (kind == "all_to_all") return CollectiveCost::all_to_all(bytes, p, s);
    if (kind == "p2p") return CollectiveCost::p2p(bytes, s);
    throw FFError("unknown collective " + kind);
  });

  // ---- cost model
  py::class_<CostModel>(m, "CostModel")
      .def(py::init<MachineSpecification>())
      .def("spec", &CostModel::spec)
      .def("load_profiles", [](CostModel& c, const std::string& s) { c.profiles().load_json(Json::parse(s)); })
      .def("put_profile", [](CostModel& c, const std::string& k, double f, double b) { c.profiles().put(k, f, b); })
      .def("profiles_json", [](CostModel& c) { return c.profiles().to_json().dump(); })
      .def("num_profiles", [](CostModel& c) { return c.profiles().size(); })
      .def_static("signature", &CostModel::signature)
      .def("op_cost",
           [](const CostModel& c, const OpAttrs& op, const std::vector<ParallelTensorShape>& ins,
              const std::vector<ParallelTensorShape>& ws, const std::vector<ParallelTensorShape>& outs, int block) {
             auto r = c.op_cost(op, ins, ws, outs, block);
             return py::make_tuple(r.forward, r.backward, r.memory, r.sync);
           })
      .def("parallel_op_cost",
           [](const CostModel& c, const OpAttrs& op, const ParallelTensorShape& in, const ParallelTensorShape& out,
              int block) {
             auto r = c.parallel_op_cost(op, in, out, block);
             return py::make_tuple(r.forward, r.backward, r.memory, r.sync);
           })
      .def("pcg_node_cost", [](const CostModel& c, const ParallelComputationGraph& p, int node, int block) {
        auto r = pcg_node_cost(c, p, node, block);
        return py::make_tuple(r.forward, r.backward, r.memory, r.sync);
      });

  // ---- SP decomposition
  m.def("sp_decomposition", [](const ParallelComputationGraph& p, bool strict) -> py::object {
    auto g = data_path_digraph(p);
    if (strict) {
      auto t = get_series_parallel_decomposition(g);
      if (!t) return py::none();
      return py::str(t->to_json().dump());
    }
    return py::str(get_relaxed_sp_decomposition(g).to_json().dump());
  }, py::arg("pcg"), py::arg("strict") = false);
  m.def("cg_sp_decomposition", [](const ComputationGraph& cg, bool strict) -> py::object {
    // reference CG path: plain SP first; fall back by dropping weights (implicit in leaves)
    DiGraph g = cg.g.digraph();
    auto t = get_series_parallel_decomposition(g);
    if (!t) {
      std::set<int> keep;
      for (int id : g.nodes)
        if (cg.g.node(id).label.op.type != OpType::WEIGHT) keep.insert(id);
      g = g.induced_subgraph(keep);
      t = get_series_parallel_decomposition(g);
    }
    if (t) return py::str(t->to_json().dump());
    if (strict) return py::none();
    return py::str(get_relaxed_sp_decomposition(g).to_json().dump());
  }, py::arg("cg"), py::arg("strict") = false);
  m.def("digraph_sp_decomposition", [](const std::vector<std::pair<int, int>>& edges, const std::vector<int>& nodes,
                                       bool strict) -> py::object {
    DiGraph g;
    for (int n : nodes) g.add_node(n);
    for (auto const& e : edges) g.add_edge(e.first, e.second);
    if (strict) {
      auto t = get_series_parallel_decomposition(g);
      if (!t) return py::none();
      return py::str(t->to_json().dump());
    }
    return py::str(get_relaxed_sp_decomposition(g).to_json().dump());
  }, py::arg("edges"), py::arg("nodes") = std::vector<int>{}, py::arg("strict") = true);

  // ---- per-layer configs and lowering
  m.def("candidate_configs", [](const ComputationGraph& cg, int node, int world, bool pp, bool ap, bool partial) {
    SearchSpaceOptions o;
    o.enable_parameter_parallel = pp;
    o.enable_attribute_parallel = ap;
    o.allow_partial_world = partial;
    std::vector<std::string> r;
    for (auto const& c : candidate_configs(cg, node, world, o)) r.push_back(c.to_json().dump());
    return r;
  }, py::arg("cg"), py::arg("node"), py::arg("world"), py::arg("enable_parameter_parallel") = true,
        py::arg("enable_attribute_parallel") = false, py::arg("allow_partial_world") = false);
  m.def("data_parallel_strategy", [](const ComputationGraph& cg, int world) {
    return strategy_to_json(cg, data_parallel_strategy(cg, world)).dump();
  });
  m.def("lower_strategy", [](const ComputationGraph& cg, const std::string& strategy, int world) {
    auto L = lower_strategy(cg, strategy_from_json(cg, Json::parse(strategy)), world);
    return py::make_tuple(L.pcg, L.cg_to_pcg, L.num_parallel_ops);
  });
  m.def("convert_parallel_shape", [](ParallelComputationGraph& p, ValueRef v, const ParallelTensorShape& t) {
    int n = 0;
    auto r = convert_parallel_shape(p, v, t, &n);
    return py::make_tuple(r, n);
  });

  // ---- liveness memory plan (ff/memory_plan.h): JSON list, one per device
  m.def("plan_memory", [](const ParallelComputationGraph& p, const std::map<int, std::vector<int>>& views, int world,
                          bool training, double weight_bytes_per_param, bool with_blocks,
                          const std::map<int, double>& live_copies, double act_elem_bytes, bool executor_fusions) {
    MemoryPlanConfig c;
    c.training = training;
    c.weight_bytes_per_param = weight_bytes_per_param;
    c.live_copies = live_copies;
    c.act_elem_bytes = act_elem_bytes;
    c.executor_fusions = executor_fusions;
    Json a = Json::array();
    for (auto const& pl : plan_memory(p, std::map<int, Placement>(views.begin(), views.end()), world, c))
      a.push_back(pl.to_json(with_blocks));
    return a.dump();
  }, py::arg("pcg"), py::arg("views") = std::map<int, std::vector<int>>{}, py::arg("world") = 1,
        py::arg("training") = true, py::arg("weight_bytes_per_param") = 16.0, py::arg("with_blocks") = false,
        py::arg("live_copies") = std::map<int, double>{}, py::arg("act_elem_bytes") = 0.0,
        py::arg("executor_fusions") = false);

  // ---- simulator
  m.def("simulate", [](const ParallelComputationGraph& p, const CostModel& cm, const std::string& sim_cfg,
                       const std::map<int, std::vector<int>>& views, bool dot, const NetworkModel* net) {
    SimConfig c = sim_config_from_json(sim_cfg.empty() ? Json::object() : Json::parse(sim_cfg));
    c.network = net;
    Simulator S(cm, c);
    auto r = S.simulate(p, std::map<int, Placement>(views.begin(), views.end()), dot);
    Json j = r.to_json();
    if (dot) {
      Json tl = Json::array();
      for (auto const& t : r.tasks) {
        Json x = Json::object();
        x["type"] = static_cast<int64_t>(t.type);
        x["name"] = t.name;
        x["devices"] = Json(std::vector<int64_t>(t.devices.begin(), t.devices.end()));
        x["src"] = static_cast<int64_t>(t.src);
        x["dst"] = static_cast<int64_t>(t.dst);
        x["bytes"] = t.bytes;
        x["links"] = Json(std::vector<int64_t>(t.links.begin(), t.links.end()));
        x["start"] = t.start_time;
        x["end"] = t.end_time;
        x["deps"] = Json(std::vector<int64_t>(t.deps.begin(), t.deps.end()));
        tl.push_back(x);
      }
      j["tasks"] = tl;
    }
    return py::make_tuple(j.dump(), dot ? S.task_graph_dot(r) : std::string());
  }, py::arg("pcg"), py::arg("cost_model"), py::arg("sim_config") = "",
        py::arg("views") = std::map<int, std::vector<int>>{}, py::arg("dot") = false,
        py::arg("network") = static_cast<const NetworkModel*>(nullptr));
  m.def("region_transfers", [](const ParallelTensorShape& t, const std::vector<int>& src, const std::vector<int>& dst) {
    return region_transfers(t, src, dst);
  });
  m.def("evaluate_strategy", [](const ComputationGraph& cg, const std::string& strategy, const CostModel& cm,
                                const std::string& sim_cfg, int world) {
    SimResult r;
    double t = evaluate_strategy(cg, strategy_from_json(cg, Json::parse(strategy)), cm,
                                 sim_config_from_json(sim_cfg.empty() ? Json::object() : Json::parse(sim_cfg)),
                                 world, &r);
    return py::make_tuple(t, r.to_json().dump());
  });

  // ---- machine mapping
  m.def("machine_mapping", [](const ParallelComputationGraph& p, const CostModel& cm, int world, bool contiguous) {
    MachineMappingOptions o;
    o.contiguous_only = contiguous;
    MachineMappingResult r;
    {
      py::gil_scoped_release nogil;
      r = get_optimal_machine_mapping(p, cm, world, o);
    }
    return py::make_tuple(r.runtime, r.feasible, views_to_py(r.views), r.to_json().dump());
  }, py::arg("pcg"), py::arg("cost_model"), py::arg("world"), py::arg("contiguous_only") = false);
  m.def("mm_subtree_signatures", [](const ParallelComputationGraph& p) {
    return get_machine_mapping_problem_tree(p).tree.signatures();
  });
  // map several PCGs in turn through ONE mapping cache (the joint search's
  // shared MachineMappingCache): per PCG (runtime, cache entries, hits so far)
  m.def("machine_mapping_sequence", [](const std::vector<ParallelComputationGraph>& ps, const CostModel& cm,
                                       int world) {
    MMCache cache;
    std::vector<std::tuple<double, int64_t, int64_t>> out;
    for (auto const& p : ps) {
      auto r = get_optimal_machine_mapping(p, cm, world, MachineMappingOptions{}, &cache);
      out.emplace_back(r.runtime, static_cast<int64_t>(cache.results.size()), static_cast<int64_t>(cache.hits));
    }
    return out;
  });
  m.def("machine_mapping_problem_tree", [](const ParallelComputationGraph& p) {
    auto prob = get_machine_mapping_problem_tree(p);
    Json j = Json::object();
    j["num_entries"] = static_cast<int64_t>(prob.tree.e.size());
    int series = 0, parallel = 0, moves = 0;
    for (auto const& e : prob.tree.e) {
      series += e.kind == MMProblemTree::SERIES;
      parallel += e.kind == MMProblemTree::PARALLEL;
      moves += static_cast<int>(e.movement.size());
    }
    j["series"] = static_cast<int64_t>(series);
    j["parallel"] = static_cast<int64_t>(parallel);
    j["movements"] = static_cast<int64_t>(moves);
    Json leaves = Json::object();
    for (auto const& kv : prob.node_of_path) leaves[path_to(kv.first)] = static_cast<int64_t>(kv.second);
    j["leaves"] = leaves;
    return j.dump();
  });
  // generic DP on a JSON problem + table costs (tests: the reference cases)
  m.def("machine_mapping_dp", [](const std::string& problem, const std::string& table, const std::string& allowed,
                                 const std::string& resources) {
    MMProblemTree t;
    t.root = tree_from_json(t, Json::parse(problem));
    TableEstimator est;
    Json tj = Json::parse(table);
    for (auto const& x : tj.at("ops").as_array())
      est.ops.emplace(x.at("leaf").as_string() + "@" + MachineView::from_json(x.at("view")).str(), x.at("cost").as_double());
    for (auto const& x : tj.at("movements").as_array()) {
      std::vector<SingleTensorMovement> mv;
      for (auto const& y : x.at("tensors").as_array()) {
        SingleTensorMovement s;
        for (auto const& v : y.at("src").as_array()) s.src.push_back(MachineView::from_json(v));
        for (auto const& v : y.at("dst").as_array()) s.dst.push_back(MachineView::from_json(v));
        mv.push_back(s);
      }
      est.moves.emplace(TableEstimator::move_key(mv), x.at("cost").as_double());  // first wins (unordered_map init)
    }
    std::vector<std::pair<MachineResource, std::vector<MachineView>>> allow;
    const Json aj = Json::parse(allowed);
    for (auto const& x : aj.as_array()) {
      std::vector<MachineView> vs;
      for (auto const& v : x.at("views").as_array()) vs.push_back(MachineView::from_json(v));
      allow.push_back({resource_from(x.at("resource")), vs});
    }
    MMContext ctx;
    ctx.cost = &est;
    ctx.allowed_views = [&](const UnmappedOpKey&, const MachineResource& r) {
      for (auto const& a : allow)
        if (a.first.num_nodes == r.num_nodes && a.first.gpus_per_node == r.gpus_per_node) return a.second;
      return std::vector<MachineView>{};
    };
    MMCache cache;
    auto r = get_optimal_machine_mapping(cache, ctx, t, resource_from(Json::parse(resources)));
    if (!r) return std::string("null");
    Json j = Json::object();
    j["runtime"] = r->runtime;
    Json m = Json::object();
    for (auto const& kv : r->mapping) m[path_to(kv.first)] = kv.second.to_json();
    j["mapping"] = m;
    j["cache_entries"] = static_cast<int64_t>(cache.results.size());
    return j.dump();
  });
  // machine-mapping result combinators on JSON results: null = infeasible,
  // {"runtime": r, "mapping": {"LR..": view}} (paths as in machine_mapping_dp)
  auto mm_from = [](const std::string& s) -> MMResult {
    Json j = Json::parse(s);
    if (j.is_null()) return std::nullopt;
    FeasibleMachineMapping f;
    f.runtime = j.at("runtime").as_double();
    if (j.contains("mapping"))
      for (auto const& kv : j.at("mapping").as_object()) {
        BinaryTreePath p;
        for (char c : kv.first) p.push_back(c == 'R' ? 1 : 0);
        f.mapping[p] = MachineView::from_json(kv.second);
      }
    return f;
  };
  auto mm_to = [](const MMResult& r) -> std::string {
    if (!r) return "null";
    Json j = Json::object();
    j["runtime"] = r->runtime;
    Json m = Json::object();
    for (auto const& kv : r->mapping) m[path_to(kv.first)] = kv.second.to_json();
    j["mapping"] = m;
    return j.dump();
  };
  m.def("mm_series_combine", [=](double comm, const std::string& pre, const std::string& post, bool r_then_l) {
    return mm_to(series_combine(comm, mm_from(pre), mm_from(post), r_then_l));
  }, py::arg("comm"), py::arg("pre"), py::arg("post"), py::arg("r_then_l") = false);
  m.def("mm_parallel_combine", [=](const std::string& l, const std::string& r) {
    return mm_to(parallel_combine(mm_from(l), mm_from(r)));
  });
  m.def("mm_minimize_runtime", [=](const std::string& a, const std::string& b) {
    return mm_to(minimize_runtime(mm_from(a), mm_from(b)));
  });
  m.def("machine_resource_splits", [](const std::string& resource) {
    Json out = Json::array();
    for (auto const& sp : get_machine_resource_splits(resource_from(Json::parse(resource)))) {
      Json x = Json::array();
      for (auto const* r : {&sp.first, &sp.second}) {
        Json y = Json::object();
        y["node_offset"] = static_cast<int64_t>(r->node_offset);
        y["num_nodes"] = static_cast<int64_t>(r->num_nodes);
        y["gpu_offset"] = static_cast<int64_t>(r->gpu_offset);
        y["gpus_per_node"] = static_cast<int64_t>(r->gpus_per_node);
        x.push_back(y);
      }
      out.push_back(x);
    }
    return out.dump();
  });

  // ---- substitutions
  py::class_<Substitution>(m, "Substitution")
      .def_readonly("name", &Substitution::name)
      .def("num_pattern_nodes", [](const Substitution& s) { return s.pattern.nodes.size(); })
      .def("num_output_nodes", [](const Substitution& s) { return s.out_nodes.size(); })
      .def("to_json", [](const Substitution& s) { return s.to_json().dump(); });
  m.def("generate_parallelization_substitutions", &generate_parallelization_substitutions);
  m.def("find_pattern_matches", [](const Substitution& s, const ParallelComputationGraph& p, size_t max) {
    std::vector<std::pair<std::vector<int>, std::vector<ValueRef>>> r;
    for (auto const& mt : find_pattern_matches(s.pattern, p, max)) r.push_back({mt.node_map, mt.input_map});
    return r;
  }, py::arg("sub"), py::arg("pcg"), py::arg("max_matches") = 4096);
  m.def("apply_substitution", [](const ParallelComputationGraph& p, const Substitution& s,
                                 const std::vector<int>& node_map, const std::vector<ValueRef>& input_map) -> py::object {
    PCGPatternMatch mt{node_map, input_map};
    auto r = apply_substitution(p, s, mt);
    if (!r) return py::none();
    return py::cast(*r);
  });

  py::class_<LegacyRuleCollection>(m, "LegacyRuleCollection")
      .def("__len__", [](const LegacyRuleCollection& c) { return c.rules.size(); })
      .def("name", [](const LegacyRuleCollection& c, size_t i) { return c.rules.at(i).name; })
      .def("op_types", [](const LegacyRuleCollection& c, size_t i) {
        std::vector<std::string> src, dst;
        for (auto const& o : c.rules.at(i).src) src.push_back(o.type);
        for (auto const& o : c.rules.at(i).dst) dst.push_back(o.type);
        return py::make_tuple(src, dst);
      })
      .def("to_dot", [](const LegacyRuleCollection& c, size_t i) { return legacy_rule_to_dot(c.rules.at(i)); })
      .def("to_substitution", [](const LegacyRuleCollection& c, size_t i) -> py::object {
        auto s = substitution_from_legacy_rule(c.rules.at(i));
        if (!s) return py::none();
        return py::cast(*s);
      })
      .def("conversion_failure", [](const LegacyRuleCollection& c, size_t i) {
        std::string why;
        auto s = substitution_from_legacy_rule(c.rules.at(i), &why);
        return s ? std::string() : why;
      });
  m.def("load_substitutions", [](const std::string& s) {
    std::vector<std::string> skipped;
    auto subs = load_substitutions(Json::parse(s), &skipped);
    return py::make_tuple(subs, skipped);
  });
  // value-semantics round trips (tests/test_ir_properties.py)
  m.def("machine_view_roundtrip", [](const std::string& s) {
    const MachineView v = MachineView::from_json(Json::parse(s));
    return v.to_json().dump();
  });
  m.def("layer_config_roundtrip", [](const std::string& s) { return LayerConfig::from_json(Json::parse(s)).to_json().dump(); });
  m.def("substitution_from_json", [](const std::string& s) { return Substitution::from_json(Json::parse(s)); });
  m.def("load_legacy_rules", [](const std::string& s) { return load_legacy_rules(Json::parse(s)); });

  // ---- model zoo (C++ CG builders)
  m.def("model_names", &model_names);
  m.def("get_model_computation_graph", [](const std::string& name, const std::string& cfg) {
    return get_model_computation_graph(name, cfg.empty() ? Json::object() : Json::parse(cfg));
  }, py::arg("name"), py::arg("config") = "");

  // ---- search
  m.def("mcmc_search", [](const ComputationGraph& cg, const CostModel& cm, const std::string& cfg) {
    SearchResult r;
    {
      py::gil_scoped_release nogil;
      r = mcmc_search(cg, cm, search_config_from_json(Json::parse(cfg)));
    }
    return py::make_tuple(r.pcg, r.to_json(&cg).dump(), views_to_py(r.views));
  });
  m.def("unity_search", [](const ParallelComputationGraph& p, const CostModel& cm, const std::string& cfg) {
    SearchResult r;
    {
      py::gil_scoped_release nogil;
      r = unity_search(p, cm, search_config_from_json(Json::parse(cfg)));
    }
    return py::make_tuple(r.pcg, r.to_json().dump(), views_to_py(r.views));
  });
  m.def("graph_optimize", [](const ComputationGraph& cg, const CostModel& cm, const std::string& cfg) {
    SearchResult r;
    {
      py::gil_scoped_release nogil;
      r = graph_optimize(cg, cm, search_config_from_json(Json::parse(cfg)));
    }
    return py::make_tuple(r.pcg, r.to_json(&cg).dump(), views_to_py(r.views));
  });
}

}  // namespace ff
