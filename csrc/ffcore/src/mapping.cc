#include "ff/mapping.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <sstream>

namespace ff {

static constexpr double kInf = std::numeric_limits<double>::infinity();

static std::string path_str(const BinaryTreePath& p) {
  std::string s;
  for (int x : p) s += x ? 'R' : 'L';
  return s.empty() ? "." : s;
}

// ---------------------------------------------------------------------------
// problem tree
std::vector<int> UnmappedOpKey::task_space() const {
  if (outputs.empty()) return {1};
  return operator_task_space(outputs[0]);
}

int MMProblemTree::add_leaf(UnmappedOpKey k) {
  Entry x;
  x.kind = LEAF;
  x.leaf = std::move(k);
  e.push_back(std::move(x));
  return static_cast<int>(e.size()) - 1;
}
int MMProblemTree::add_series(std::vector<AbstractedSingleTensorMovement> m, int l, int r) {
  Entry x;
  x.kind = SERIES;
  x.left = l;
  x.right = r;
  x.movement = std::move(m);
  e.push_back(std::move(x));
  return static_cast<int>(e.size()) - 1;
}
int MMProblemTree::add_parallel(int l, int r) {
  Entry x;
  x.kind = PARALLEL;
  x.left = l;
  x.right = r;
  e.push_back(std::move(x));
  return static_cast<int>(e.size()) - 1;
}
std::vector<BinaryTreePath> MMProblemTree::leaf_paths(int idx) const {
  std::vector<BinaryTreePath> out;
  BinaryTreePath cur;
  std::function<void(int)> rec = [&](int i) {
    if (e[i].kind == LEAF) {
      out.push_back(cur);
      return;
    }
    cur.push_back(0);
    rec(e[i].left);
    cur.back() = 1;
    rec(e[i].right);
    cur.pop_back();
  };
  if (idx >= 0) rec(idx);
  return out;
}
int MMProblemTree::subtree_at(int idx, const BinaryTreePath& path) const {
  int i = idx;
  for (int step : path) {
    if (i < 0 || e[i].kind == LEAF) return -1;
    i = step == 0 ? e[i].left : e[i].right;
  }
  return i;
}

bool MachineResource::operator<(const MachineResource& o) const {
  if (node_offset != o.node_offset) return node_offset < o.node_offset;
  if (num_nodes != o.num_nodes) return num_nodes < o.num_nodes;
  if (gpu_offset != o.gpu_offset) return gpu_offset < o.gpu_offset;
  return gpus_per_node < o.gpus_per_node;
}
std::string MachineResource::str() const {
  return std::to_string(node_offset) + "+" + std::to_string(num_nodes) + "x" + std::to_string(gpu_offset) + "+" +
         std::to_string(gpus_per_node);
}

std::vector<std::pair<MachineResource, MachineResource>> get_machine_resource_splits(const MachineResource& r) {
  std::vector<std::pair<MachineResource, MachineResource>> out;
  auto add = [&](const MachineResource& a, const MachineResource& b) {
    for (auto const& x : out)
      if (x.first == a && x.second == b) return;
    out.push_back({a, b});
  };
  for (int i = 1; i < r.num_nodes; i *= 2)
    for (int first : {i, r.num_nodes - i}) {
      MachineResource a = r, b = r;
      a.num_nodes = first;
      b.node_offset = r.node_offset + first;
      b.num_nodes = r.num_nodes - first;
      add(a, b);
    }
  for (int i = 1; i < r.gpus_per_node; i *= 2)
    for (int first : {i, r.gpus_per_node - i}) {
      MachineResource a = r, b = r;
      a.gpus_per_node = first;
      b.gpu_offset = r.gpu_offset + first;
      b.gpus_per_node = r.gpus_per_node - first;
      add(a, b);
    }
  return out;
}

std::vector<MachineView> get_allowed_machine_views(const std::vector<int>& ts, const MachineResource& r,
                                                   const MachineSpecification& spec) {
  MachineSpecification sub = spec;
  sub.num_nodes = r.num_nodes;
  sub.num_gpus_per_node = r.gpus_per_node;
  auto views = get_allowed_machine_views(ts, sub);
  for (auto& v : views) {
    v.start.node_idx += r.node_offset;
    v.start.device_idx += r.gpu_offset;
  }
  return views;
}

// ---------------------------------------------------------------------------
// constraints and results
std::string MachineMappingConstraints::key() const {
  std::string s;
  for (auto const& kv : views) {
    s += path_str(kv.first);
    s += '=';
    s += kv.second ? kv.second->str() : "-";
    s += ';';
  }
  return s;
}

MachineMappingConstraints get_unconstrained_solution_for_layers(const std::vector<BinaryTreePath>& layers) {
  MachineMappingConstraints c;
  for (auto const& p : layers) c.views[p] = std::nullopt;
  return c;
}

MachineMappingConstraints restrict_to_child(const MachineMappingConstraints& c, int child) {
  MachineMappingConstraints r;
  for (auto const& kv : c.views)
    if (!kv.first.empty() && kv.first[0] == child) r.views[BinaryTreePath(kv.first.begin() + 1, kv.first.end())] = kv.second;
  return r;
}

std::optional<MachineMappingConstraints> with_additional_constraints(const MachineMappingConstraints& c,
                                                                    const ObliviousMapping& extra) {
  MachineMappingConstraints r = c;
  for (auto const& kv : extra) {
    auto it = r.views.find(kv.first);
    if (it == r.views.end() || !it->second) r.views[kv.first] = kv.second;
    else if (*it->second != kv.second) return std::nullopt;
  }
  return r;
}

static ObliviousMapping binary_combine(const ObliviousMapping& l, const ObliviousMapping& r) {
  ObliviousMapping m;
  for (auto const& kv : l) {
    BinaryTreePath p{0};
    p.insert(p.end(), kv.first.begin(), kv.first.end());
    m[p] = kv.second;
  }
  for (auto const& kv : r) {
    BinaryTreePath p{1};
    p.insert(p.end(), kv.first.begin(), kv.first.end());
    m[p] = kv.second;
  }
  return m;
}

MMResult series_combine(double comm, const MMResult& pre, const MMResult& post, bool r_then_l) {
  if (!pre || !post || !std::isfinite(comm)) return std::nullopt;
  FeasibleMachineMapping r;
  r.runtime = pre->runtime + comm + post->runtime;
  r.mapping = r_then_l ? binary_combine(post->mapping, pre->mapping) : binary_combine(pre->mapping, post->mapping);
  return r;
}

MMResult parallel_combine(const MMResult& l, const MMResult& r) {
  if (!l || !r) return std::nullopt;
  FeasibleMachineMapping x;
  x.runtime = std::max(l->runtime, r->runtime);
  x.mapping = binary_combine(l->mapping, r->mapping);
  return x;
}

MMResult minimize_runtime(const MMResult& a, const MMResult& b) {
  if (!a) return b;
  if (!b) return a;
  return b->runtime < a->runtime ? b : a;
}

// ---------------------------------------------------------------------------
// subtree signatures (content keys of the shared cache)
namespace {
uint64_t fnv(const std::string& s, uint64_t h) {
  for (unsigned char ch : s) {
    h ^= ch;
    h *= 1099511628211ull;
  }
  return h;
}
std::string pshape_str(const ParallelTensorShape& p) { return p.to_json().dump(); }
std::string paths_str(const std::set<BinaryTreePath>& ps) {
  std::string s;
  for (auto const& p : ps) {
    s += "[";
    for (int x : p) s += std::to_string(x) + ",";
    s += "]";
  }
  return s;
}
}  // namespace

std::vector<std::string> MMProblemTree::signatures() const {
  std::vector<std::string> out(e.size());
  std::vector<std::string> text(e.size());
  // children are added before their parents (add_series / add_parallel take
  // existing indices), so one forward pass sees every child first
  for (size_t i = 0; i < e.size(); ++i) {
    auto const& x = e[i];
    std::string d;
    if (x.kind == LEAF) {
      d = "L" + x.leaf.op.to_json().dump() + "#" + x.leaf.id;
      for (auto const& v : x.leaf.inputs) d += "i" + pshape_str(v);
      for (auto const& v : x.leaf.weights) d += "w" + pshape_str(v);
      for (auto const& v : x.leaf.outputs) d += "o" + pshape_str(v);
    } else {
      d = (x.kind == SERIES ? "S(" : "P(") + out[x.left] + "," + out[x.right] + ")";
      for (auto const& m : x.movement) d += "m" + pshape_str(m.shape) + paths_str(m.src) + ">" + paths_str(m.dst);
    }
    char buf[40];
    snprintf(buf, sizeof(buf), "%016llx%016llx", static_cast<unsigned long long>(fnv(d, 1469598103934665603ull)),
             static_cast<unsigned long long>(fnv(d, 0x9e3779b97f4a7c15ull)));
    out[i] = buf;
  }
  return out;
}

// ---------------------------------------------------------------------------
// the DP
namespace {

struct Solver {
  MMCache& cache;
  const MMContext& ctx;
  const MMProblemTree& t;
  std::vector<std::string> sig = t.signatures();

  MMResult solve(int idx, const MachineResource& res, const MachineMappingConstraints& c) {
    std::string key = sig[idx] + "@" + res.str() + "|" + c.key();
    auto it = cache.results.find(key);
    if (it != cache.results.end()) {
      ++cache.hits;
      return it->second;
    }
    ++cache.misses;
    MMResult r;
    auto const& e = t.e[idx];
    if (e.kind == MMProblemTree::LEAF) r = leaf(e, res, c);
    else if (e.kind == MMProblemTree::SERIES) r = series(e.movement, e.left, e.right, res, c, false);
    else r = parallel(e, res, c);
    cache.results.emplace(std::move(key), r);
    return r;
  }

  MMResult leaf(const MMProblemTree::Entry& e, const MachineResource& res, const MachineMappingConstraints& c) {
    std::vector<MachineView> cands = ctx.allowed_views(e.leaf, res);
    auto it = c.views.find(BinaryTreePath{});
    if (it != c.views.end() && it->second) {
      // a view an enclosing series split fixed: feasible only where these
      // resources allow it (a resource split below that split may not)
      if (std::find(cands.begin(), cands.end(), *it->second) == cands.end()) return std::nullopt;
      cands = {*it->second};
    }
    MMResult best;
    for (auto const& v : cands) {
      double cost = ctx.cost->estimate_op(e.leaf, v);
      if (!std::isfinite(cost)) continue;
      FeasibleMachineMapping f;
      f.runtime = cost;
      f.mapping[BinaryTreePath{}] = v;
      best = minimize_runtime(best, f);
    }
    return best;
  }

  // every assignment of views to `layers` (paths relative to subtree `sub`)
  std::vector<ObliviousMapping> assignments(int sub, const std::set<BinaryTreePath>& layers,
                                            const MachineMappingConstraints& c, const MachineResource& res) {
    std::vector<BinaryTreePath> ls(layers.begin(), layers.end());
    std::vector<std::vector<MachineView>> opts;
    for (auto const& p : ls) {
      auto it = c.views.find(p);
      if (it != c.views.end() && it->second) {
        opts.push_back({*it->second});
        continue;
      }
      int leaf = t.subtree_at(sub, p);
      if (leaf < 0 || t.e[leaf].kind != MMProblemTree::LEAF) throw FFError("machine mapping: bad boundary path");
      opts.push_back(ctx.allowed_views(t.e[leaf].leaf, res));
    }
    // cap the product: keep each layer's cheapest views until it fits
    auto product = [&]() {
      double n = 1;
      for (auto const& o : opts) n *= static_cast<double>(o.size());
      return n;
    };
    if (product() > static_cast<double>(ctx.max_boundary_assignments)) {
      for (size_t k = 0; k < ls.size(); ++k) {
        int leaf = t.subtree_at(sub, ls[k]);
        auto& o = opts[k];
        std::stable_sort(o.begin(), o.end(), [&](const MachineView& a, const MachineView& b) {
          return ctx.cost->estimate_op(t.e[leaf].leaf, a) < ctx.cost->estimate_op(t.e[leaf].leaf, b);
        });
      }
      while (product() > static_cast<double>(ctx.max_boundary_assignments)) {
        size_t widest = 0;
        for (size_t k = 1; k < opts.size(); ++k)
          if (opts[k].size() > opts[widest].size()) widest = k;
        if (opts[widest].size() <= 1) break;
        opts[widest].resize(std::max<size_t>(1, opts[widest].size() / 2));
      }
    }
    std::vector<ObliviousMapping> out{ObliviousMapping{}};
    for (size_t k = 0; k < ls.size(); ++k) {
      std::vector<ObliviousMapping> next;
      for (auto const& m : out)
        for (auto const& v : opts[k]) {
          auto x = m;
          x[ls[k]] = v;
          next.push_back(std::move(x));
        }
      out.swap(next);
    }
    return out;
  }

  MMResult series(const std::vector<AbstractedSingleTensorMovement>& mv, int l, int r, const MachineResource& res,
                  const MachineMappingConstraints& c, bool r_then_l) {
    std::set<BinaryTreePath> src, dst;
    for (auto const& m : mv) {
      src.insert(m.src.begin(), m.src.end());
      dst.insert(m.dst.begin(), m.dst.end());
    }
    const auto lc = restrict_to_child(c, 0), rc = restrict_to_child(c, 1);
    auto pre_as = assignments(l, src, lc, res);
    auto post_as = assignments(r, dst, rc, res);
    std::vector<MMResult> post_rs;
    for (auto const& pa : post_as) {
      auto cc = with_additional_constraints(rc, pa);
      post_rs.push_back(cc ? solve(r, res, *cc) : MMResult{});
    }
    MMResult best;
    for (auto const& pre : pre_as) {
      auto cc = with_additional_constraints(lc, pre);
      if (!cc) continue;
      MMResult pre_r = solve(l, res, *cc);
      if (!pre_r) continue;
      for (size_t k = 0; k < post_as.size(); ++k) {
        if (!post_rs[k]) continue;
        std::vector<SingleTensorMovement> concrete;
        for (auto const& m : mv) {
          SingleTensorMovement s;
          s.shape = m.shape;
          for (auto const& p : m.src) {
            s.src.push_back(pre.at(p));
            s.src_task_spaces.push_back(t.e[t.subtree_at(l, p)].leaf.task_space());
          }
          for (auto const& p : m.dst) {
            s.dst.push_back(post_as[k].at(p));
            s.dst_task_spaces.push_back(t.e[t.subtree_at(r, p)].leaf.task_space());
          }
          concrete.push_back(std::move(s));
        }
        const double comm = concrete.empty() ? 0.0 : ctx.cost->estimate_movement(concrete);
        best = minimize_runtime(best, series_combine(comm, pre_r, post_rs[k], r_then_l));
      }
    }
    return best;
  }

  MMResult parallel(const MMProblemTree::Entry& e, const MachineResource& res, const MachineMappingConstraints& c) {
    MMResult best = series({}, e.left, e.right, res, c, false);
    const auto lc = restrict_to_child(c, 0), rc = restrict_to_child(c, 1);
    for (auto const& sp : get_machine_resource_splits(res)) {
      MMResult a = solve(e.left, sp.first, lc);
      if (!a) continue;
      MMResult b = solve(e.right, sp.second, rc);
      best = minimize_runtime(best, parallel_combine(a, b));
    }
    return best;
  }
};

}  // namespace

MMResult get_optimal_machine_mapping(MMCache& cache, const MMContext& ctx, const MMProblemTree& tree, int idx,
                                     const MachineResource& resources, const MachineMappingConstraints& constraints) {
  if (!ctx.cost || !ctx.allowed_views) throw FFError("machine mapping: incomplete context");
  Solver s{cache, ctx, tree};
  return s.solve(idx, resources, constraints);
}

MMResult get_optimal_machine_mapping(MMCache& cache, const MMContext& ctx, const MMProblemTree& tree,
                                     const MachineResource& resources) {
  if (tree.root < 0) return FeasibleMachineMapping{};
  return get_optimal_machine_mapping(cache, ctx, tree, tree.root, resources,
                                     get_unconstrained_solution_for_layers(tree.leaf_paths(tree.root)));
}

// ---------------------------------------------------------------------------
// PCG adapter
PCGMappingProblem get_machine_mapping_problem_tree(const ParallelComputationGraph& pcg) {
  PCGMappingProblem out;
  auto sp = get_relaxed_sp_decomposition(data_path_digraph(pcg));
  if (sp.root < 0) return out;
  auto roles = classify_nodes(pcg);
  // returns the problem-tree index; `paths`: PCG node -> path inside this subtree
  std::function<int(int, std::map<int, BinaryTreePath>&)> conv = [&](int i, std::map<int, BinaryTreePath>& paths) {
    auto const& e = sp.e[i];
    if (e.kind == SPTree::LEAF) {
      UnmappedOpKey k;
      const int n = e.node;
      auto const& nd = pcg.g.node(n);
      k.op = nd.label.op;
      k.node = n;
      for (auto const& v : pcg.layer_data_inputs(n)) k.inputs.push_back(pcg.shape(v));
      for (auto const& v : pcg.layer_weights(n)) k.weights.push_back(pcg.shape(v));
      for (auto const& o : nd.outputs) k.outputs.push_back(o.shape);
      paths[n] = BinaryTreePath{};
      return out.tree.add_leaf(std::move(k));
    }
    std::map<int, BinaryTreePath> lp, rp;
    int l = conv(e.left, lp);
    int r = conv(e.right, rp);
    int idx;
    if (e.kind == SPTree::SERIES) {
      // every tensor a left leaf produces and a right leaf consumes (skip
      // connections included; each edge is priced at its lowest common split)
      std::map<ValueRef, AbstractedSingleTensorMovement> mv;
      for (auto const& kv : rp) {
        for (auto const& v : pcg.g.node(kv.first).inputs) {
          auto it = lp.find(v.node);
          if (it == lp.end() || roles.at(v.node) == NodeRole::WEIGHT_PATH) continue;
          auto& m = mv[v];
          m.shape = pcg.shape(v);
          m.src.insert(it->second);
          m.dst.insert(kv.second);
        }
      }
      std::vector<AbstractedSingleTensorMovement> list;
      for (auto& kv : mv) list.push_back(std::move(kv.second));
      idx = out.tree.add_series(std::move(list), l, r);
    } else {
      idx = out.tree.add_parallel(l, r);
    }
    for (auto const& kv : lp) {
      BinaryTreePath p{0};
      p.insert(p.end(), kv.second.begin(), kv.second.end());
      paths[kv.first] = p;
    }
    for (auto const& kv : rp) {
      BinaryTreePath p{1};
      p.insert(p.end(), kv.second.begin(), kv.second.end());
      paths[kv.first] = p;
    }
    return idx;
  };
  std::map<int, BinaryTreePath> paths;
  out.tree.root = conv(sp.root, paths);
  for (auto const& kv : paths) out.node_of_path[kv.second] = kv.first;
  return out;
}

static int nodes_spanned(const Placement& p, int gpn) {
  std::set<int> n;
  for (int d : p) n.insert(d / std::max(1, gpn));
  return static_cast<int>(n.size());
}

double PCGCostEstimator::estimate_op(const UnmappedOpKey& k, const MachineView& v) const {
  if (k.node < 0) return 0.0;
  auto const& spec = cm_.spec();
  auto ts = k.task_space();
  int T = 1;
  for (int d : ts) T *= d;
  OpCost c = pcg_node_cost(cm_, pcg_, k.node, T);
  double comm_scale = 1.0;
  if (T > 1 && T <= spec.num_gpus_per_node &&
      nodes_spanned(view_placement(ts, v, spec), spec.num_gpus_per_node) > 1)
    comm_scale = spec.intra_node_bandwidth / std::max(1.0, spec.inter_node_bandwidth);
  const bool par = is_parallel_op(k.op.type);
  double t = (c.forward + c.backward) * (par ? comm_scale : 1.0);
  if (include_sync_) t += c.sync * comm_scale;
  return t;
}

double PCGCostEstimator::estimate_movement(const std::vector<SingleTensorMovement>& ms) const {
  auto const& spec = cm_.spec();
  double t = 0;
  for (auto const& m : ms) {
    if (m.src.empty()) continue;
    Placement src = view_placement(m.src_task_spaces.at(0), m.src.at(0), spec);
    for (size_t k = 0; k < m.dst.size(); ++k) {
      Placement dst = view_placement(m.dst_task_spaces.at(k), m.dst[k], spec);
      t += 2.0 * cm_.movement_cost(m.shape, src, dst);  // activation forward + gradient backward
    }
  }
  return t;
}

Json MachineMappingResult::to_json() const {
  Json j = Json::object();
  j["runtime"] = runtime;
  j["feasible"] = feasible;
  Json v = Json::object();
  for (auto const& kv : views) v[std::to_string(kv.first)] = Json(std::vector<int64_t>(kv.second.begin(), kv.second.end()));
  j["views"] = v;
  Json mv = Json::object();
  for (auto const& kv : machine_views) mv[std::to_string(kv.first)] = kv.second.to_json();
  j["machine_views"] = mv;
  j["cache_entries"] = static_cast<int64_t>(cache_entries);
  return j;
}

MachineMappingResult get_optimal_machine_mapping(const ParallelComputationGraph& pcg, const CostModel& cm, int world,
                                                 const MachineMappingOptions& opt, MMCache* shared) {
  MachineMappingResult out;
  auto const& spec = cm.spec();
  const int gpn = std::max(1, spec.num_gpus_per_node);
  MachineResource res;
  if (world <= gpn) {
    res.num_nodes = 1;
    res.gpus_per_node = world;
  } else {
    if (world % gpn) throw FFError("machine mapping: world " + std::to_string(world) + " is not whole nodes");
    res.num_nodes = world / gpn;
    res.gpus_per_node = gpn;
  }
  auto prob = get_machine_mapping_problem_tree(pcg);
  PCGCostEstimator est(pcg, cm, opt.include_sync);
  std::map<std::pair<std::vector<int>, MachineResource>, std::vector<MachineView>> view_cache;
  MMContext ctx;
  ctx.cost = &est;
  ctx.allowed_views = [&](const UnmappedOpKey& k, const MachineResource& r) -> std::vector<MachineView> {
    auto ts = k.task_space();
    auto key = std::make_pair(ts, r);
    auto it = view_cache.find(key);
    if (it != view_cache.end()) return it->second;
    auto vs = get_allowed_machine_views(ts, r, spec);
    if (opt.contiguous_only) {
      std::vector<MachineView> keep;
      for (auto const& v : vs) {
        bool ok = true;
        for (size_t i = 0; i < v.dims.size(); ++i)
          if (ts[i] > 1 && (v.dims[i].stride != 1 || v.dims[i].projection != ProjectionType::INTRA_NODE)) ok = false;
        if (ok) keep.push_back(v);
      }
      vs.swap(keep);
    }
    view_cache.emplace(key, vs);
    return vs;
  };
  MMCache local;
  MMCache& cache = shared ? *shared : local;
  MMResult r = get_optimal_machine_mapping(cache, ctx, prob.tree, res);
  out.cache_entries = cache.results.size();
  if (!r) {
    out.feasible = false;
    out.runtime = kInf;
    return out;
  }
  out.runtime = r->runtime;
  for (auto const& kv : r->mapping) {
    int n = prob.node_of_path.at(kv.first);
    int leaf = prob.tree.subtree_at(prob.tree.root, kv.first);
    out.machine_views[n] = kv.second;
    out.views[n] = view_placement(prob.tree.e[leaf].leaf.task_space(), kv.second, spec);
  }
  // weight-path nodes follow their first data-path consumer
  auto roles = classify_nodes(pcg);
  std::map<int, std::vector<int>> users;
  for (int id : pcg.g.node_ids())
    for (auto const& v : pcg.g.node(id).inputs) users[v.node].push_back(id);
  std::function<const Placement*(int)> consumer = [&](int id) -> const Placement* {
    for (int u : users[id]) {
      auto jt = out.views.find(u);
      if (jt != out.views.end() && roles.at(u) != NodeRole::WEIGHT_PATH) return &jt->second;
      if (auto p = consumer(u)) return p;
    }
    return nullptr;
  };
  Placement all = block_placement(0, world);
  for (int id : pcg.g.node_ids())
    if (roles.at(id) == NodeRole::WEIGHT_PATH) {
      auto p = consumer(id);
      out.views[id] = p ? *p : all;
    }
  return out;
}

}  // namespace ff
