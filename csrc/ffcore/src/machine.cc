#include "ff/machine.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <sstream>

namespace ff {

Json MachineSpecification::to_json() const {
  Json j = Json::object();
  j["num_nodes"] = num_nodes;
  j["num_cpus_per_node"] = num_cpus_per_node;
  j["num_gpus_per_node"] = num_gpus_per_node;
  j["inter_node_bandwidth"] = inter_node_bandwidth;
  j["intra_node_bandwidth"] = intra_node_bandwidth;
  j["peak_bf16_flops"] = peak_bf16_flops;
  j["peak_fp32_flops"] = peak_fp32_flops;
  j["mfma_efficiency"] = mfma_efficiency;
  j["hbm_bandwidth"] = hbm_bandwidth;
  j["hbm_capacity"] = hbm_capacity;
  j["kernel_launch_overhead"] = kernel_launch_overhead;
  j["collective_latency"] = collective_latency;
  j["xgmi_links"] = xgmi_links;
  j["xgmi_link_bandwidth"] = xgmi_link_bandwidth;
  j["bf16_compute"] = bf16_compute;
  auto bwmap = [](const std::map<int, double>& m) {
    Json o = Json::object();
    for (auto const& kv : m) o[std::to_string(kv.first)] = kv.second;
    return o;
  };
  if (!collective_bw.empty()) j["collective_bw"] = bwmap(collective_bw);
  if (!all_to_all_bw.empty()) j["all_to_all_bw"] = bwmap(all_to_all_bw);
  return j;
}

MachineSpecification MachineSpecification::from_json(const Json& j) {
  MachineSpecification s;
  auto gi = [&](const char* k, int& v) {
    if (j.contains(k)) v = static_cast<int>(j.at(k).as_int());
  };
  auto gd = [&](const char* k, double& v) {
    if (j.contains(k)) v = j.at(k).as_double();
  };
  gi("num_nodes", s.num_nodes);
  gi("num_cpus_per_node", s.num_cpus_per_node);
  gi("num_gpus_per_node", s.num_gpus_per_node);
  gd("inter_node_bandwidth", s.inter_node_bandwidth);
  gd("intra_node_bandwidth", s.intra_node_bandwidth);
  gd("peak_bf16_flops", s.peak_bf16_flops);
  gd("peak_fp32_flops", s.peak_fp32_flops);
  gd("mfma_efficiency", s.mfma_efficiency);
  gd("hbm_bandwidth", s.hbm_bandwidth);
  gd("hbm_capacity", s.hbm_capacity);
  gd("kernel_launch_overhead", s.kernel_launch_overhead);
  gd("collective_latency", s.collective_latency);
  gi("xgmi_links", s.xgmi_links);
  gd("xgmi_link_bandwidth", s.xgmi_link_bandwidth);
  if (j.contains("bf16_compute")) s.bf16_compute = j.at("bf16_compute").as_bool();
  for (const char* key : {"collective_bw", "all_to_all_bw"}) {
    if (!j.contains(key)) continue;
    auto& m = std::string(key) == "collective_bw" ? s.collective_bw : s.all_to_all_bw;
    for (auto const& kv : j.at(key).as_object()) m[std::stoi(kv.first)] = kv.second.as_double();
  }
  return s;
}

MachineSpecification MachineSpecification::mi355x(int num_nodes, int gpus_per_node) {
  MachineSpecification s;
  s.num_nodes = num_nodes;
  s.num_gpus_per_node = gpus_per_node;
  return s;
}

Json MachineView::to_json() const {
  Json j = Json::object();
  j["start"] = Json(std::vector<int64_t>{start.node_idx, start.device_idx});
  Json d = Json::array();
  for (auto const& x : dims) {
    Json e = Json::object();
    e["stride"] = x.stride;
    e["projection"] = x.projection == ProjectionType::INTRA_NODE ? "INTRA_NODE" : "INTER_NODE";
    d.push_back(e);
  }
  j["dimensions"] = d;
  return j;
}

MachineView MachineView::from_json(const Json& j) {
  MachineView v;
  auto st = j.at("start").as_int_vector();
  v.start = {static_cast<int>(st.at(0)), static_cast<int>(st.at(1))};
  for (auto const& e : j.at("dimensions").as_array())
    v.dims.push_back({static_cast<int>(e.at("stride").as_int()),
                      e.at("projection").as_string() == "INTER_NODE" ? ProjectionType::INTER_NODE
                                                                     : ProjectionType::INTRA_NODE});
  return v;
}

const double kMovementInfeasible = 1e30;

std::vector<int> operator_task_space(const ParallelTensorShape& out) {
  std::vector<int> ts = out.shard_degrees();
  ts.push_back(out.sum_degree);
  ts.push_back(out.discard_copy_degree);
  return ts;
}

std::optional<MachineSpaceCoordinate> get_machine_space_coordinate(const std::vector<int>& ts, const MachineView& view,
                                                                   const std::vector<int>& coord,
                                                                   const MachineSpecification& spec) {
  if (ts.size() != view.dims.size() || coord.size() != ts.size())
    throw FFError("get_machine_space_coordinate: rank mismatch");
  // per machine dimension, the task dimensions projected onto it form a mixed
  // radix with the FIRST one fastest; a dimension's digit weight is the
  // product of (degree x stride) of the earlier dimensions on the same
  // projection, times its own stride (machine_view.cc:60-81)
  MachineSpaceCoordinate r = view.start;
  int64_t coeff_node = 1, coeff_dev = 1;
  for (size_t i = 0; i < ts.size(); ++i) {
    if (coord[i] < 0 || coord[i] >= ts[i]) return std::nullopt;
    const int64_t stride = view.dims[i].stride;
    if (view.dims[i].projection == ProjectionType::INTRA_NODE) {
      r.device_idx += static_cast<int>(coeff_dev * coord[i] * stride);
      coeff_dev *= static_cast<int64_t>(ts[i]) * stride;
    } else {
      r.node_idx += static_cast<int>(coeff_node * coord[i] * stride);
      coeff_node *= static_cast<int64_t>(ts[i]) * stride;
    }
  }
  if (r.node_idx < 0 || r.node_idx >= spec.num_nodes || r.device_idx < 0 || r.device_idx >= spec.num_gpus_per_node)
    return std::nullopt;
  return r;
}

// Start-invariant views (start_invariant_machine_view.cc): the dimensions of a
// view without its start; offsets are the coordinates of the view placed at
// (0, 0), checked against the machine.
StartInvariantMachineView start_invariant_from_machine_view(const MachineView& v) { return {v.dims}; }

MachineView machine_view_from_start_invariant(const StartInvariantMachineView& s, const MachineSpaceCoordinate& start) {
  MachineView v;
  v.start = start;
  v.dims = s.dims;
  return v;
}

std::optional<MachineSpaceCoordinate> get_machine_space_offset(const std::vector<int>& ts,
                                                               const StartInvariantMachineView& s,
                                                               const std::vector<int>& coord,
                                                               const MachineSpecification& spec) {
  return get_machine_space_coordinate(ts, machine_view_from_start_invariant(s, {0, 0}), coord, spec);
}

static void for_each_coord(const std::vector<int>& ts, const std::function<void(const std::vector<int>&)>& f) {
  std::vector<int> c(ts.size(), 0);
  while (true) {
    f(c);
    int i = static_cast<int>(ts.size()) - 1;
    while (i >= 0) {
      if (++c[i] < ts[i]) break;
      c[i] = 0;
      --i;
    }
    if (i < 0) break;
  }
}

std::vector<int> get_device_ids(const std::vector<int>& ts, const MachineView& view, const MachineSpecification& spec) {
  std::vector<int> ids;
  for_each_coord(ts, [&](const std::vector<int>& c) {
    auto m = get_machine_space_coordinate(ts, view, c, spec);
    if (!m) throw FFError("get_device_ids: view " + view.str() + " does not fit the machine");
    ids.push_back(m->node_idx * spec.num_gpus_per_node + m->device_idx);
  });
  return ids;
}

std::vector<MachineView> get_allowed_machine_views(const std::vector<int>& ts, const MachineSpecification& spec) {
  std::vector<MachineView> out;
  const int n = static_cast<int>(ts.size());
  std::vector<int> nontrivial;
  for (int i = 0; i < n; ++i)
    if (ts[i] > 1) nontrivial.push_back(i);
  const int max_stride = spec.num_devices();
  // enumerate strides for the nontrivial dims (trivial dims: stride 1, intra)
  std::vector<int> strides(nontrivial.size(), 1);
  std::vector<int> projs(nontrivial.size(), 0);
  std::function<void(size_t)> rec_proj, rec_stride;
  auto emit = [&]() {
    MachineView v;
    v.dims.assign(n, MachineViewDimension{1, ProjectionType::INTRA_NODE});
    for (size_t k = 0; k < nontrivial.size(); ++k)
      v.dims[nontrivial[k]] = {strides[k], projs[k] ? ProjectionType::INTER_NODE : ProjectionType::INTRA_NODE};
    for (int node = 0; node < spec.num_nodes; ++node)
      for (int dev = 0; dev < spec.num_gpus_per_node; ++dev) {
        v.start = {node, dev};
        bool ok = true;
        std::vector<int> maxc(ts.size());
        for (int i = 0; i < n; ++i) maxc[i] = ts[i] - 1;
        // digit weights are positive, so the largest coordinate lands furthest
        if (!get_machine_space_coordinate(ts, v, maxc, spec)) ok = false;
        if (ok) {
          auto ids = get_device_ids(ts, v, spec);
          std::sort(ids.begin(), ids.end());
          if (std::adjacent_find(ids.begin(), ids.end()) != ids.end()) ok = false;  // must be injective
        }
        if (ok) out.push_back(v);
      }
  };
  rec_stride = [&](size_t k) {
    if (k == nontrivial.size()) {
      emit();
      return;
    }
    for (int s = 1; s <= max_stride; ++s) {
      strides[k] = s;
      rec_stride(k + 1);
    }
  };
  rec_proj = [&](size_t k) {
    if (k == nontrivial.size()) {
      rec_stride(0);
      return;
    }
    for (int p = 0; p < (spec.num_nodes > 1 ? 2 : 1); ++p) {
      projs[k] = p;
      rec_proj(k + 1);
    }
  };
  rec_proj(0);
  return out;
}

MachineView block_machine_view(const std::vector<int>& ts, const DeviceBlock& b, const MachineSpecification& spec) {
  int T = 1;
  for (int d : ts) T *= d;
  if (T <= 0 || b.size % T != 0) throw FFError("block_machine_view: task space does not divide the block");
  MachineView v;
  v.start = {b.start / spec.num_gpus_per_node, b.start % spec.num_gpus_per_node};
  // first dimension strided by the replica count R, the others dense above
  // it: the view covers the block exactly, R apart within each first-dim run
  const int R = b.size / T;
  for (size_t i = 0; i < ts.size(); ++i) v.dims.push_back({i == 0 ? R : 1, ProjectionType::INTRA_NODE});
  return v;
}

bool MachineView::operator<(const MachineView& o) const {
  if (start.node_idx != o.start.node_idx) return start.node_idx < o.start.node_idx;
  if (start.device_idx != o.start.device_idx) return start.device_idx < o.start.device_idx;
  if (dims.size() != o.dims.size()) return dims.size() < o.dims.size();
  for (size_t i = 0; i < dims.size(); ++i) {
    if (dims[i].stride != o.dims[i].stride) return dims[i].stride < o.dims[i].stride;
    if (dims[i].projection != o.dims[i].projection) return dims[i].projection < o.dims[i].projection;
  }
  return false;
}

std::string MachineView::str() const {
  std::string s = "(" + std::to_string(start.node_idx) + "," + std::to_string(start.device_idx) + ")[";
  for (size_t i = 0; i < dims.size(); ++i) {
    if (i) s += ",";
    s += std::to_string(dims[i].stride) + (dims[i].projection == ProjectionType::INTER_NODE ? "N" : "D");
  }
  return s + "]";
}

Placement block_placement(int start, int size) {
  Placement p(size);
  for (int i = 0; i < size; ++i) p[i] = start + i;
  return p;
}
Placement block_placement(const DeviceBlock& b) { return block_placement(b.start, b.size); }

Placement view_placement(const std::vector<int>& ts, const MachineView& v, const MachineSpecification& spec) {
  return get_device_ids(ts, v, spec);
}

std::vector<std::pair<DeviceBlock, DeviceBlock>> get_resource_splits(const DeviceBlock& b) {
  std::vector<std::pair<DeviceBlock, DeviceBlock>> out;
  for (int k = 1; k < b.size; k *= 2) {
    out.push_back({{b.start, k}, {b.start + k, b.size - k}});
    if (b.size - k != k) out.push_back({{b.start, b.size - k}, {b.start + b.size - k, k}});
  }
  return out;
}

// ---------------------------------------------------------------------------
static double eff_bw(int p, const MachineSpecification& s) {
  if (p <= 1) return 1e30;
  auto it = s.collective_bw.find(p);
  if (it != s.collective_bw.end()) return it->second;
  double links = std::min(p - 1, s.xgmi_links) * s.xgmi_link_bandwidth;
  double b = std::min(s.intra_node_bandwidth, links);
  if (p > s.num_gpus_per_node) b = std::min(b, s.inter_node_bandwidth);
  return b;
}

double CollectiveCost::all_reduce(double bytes, int p, const MachineSpecification& s) {
  if (p <= 1 || bytes <= 0) return 0;
  return 2.0 * (p - 1) / p * bytes / eff_bw(p, s) + 2.0 * (p - 1) * s.collective_latency / 4.0 + s.collective_latency;
}
double CollectiveCost::all_gather(double bytes_out, int p, const MachineSpecification& s) {
  if (p <= 1 || bytes_out <= 0) return 0;
  return (p - 1.0) / p * bytes_out / eff_bw(p, s) + s.collective_latency;
}
double CollectiveCost::reduce_scatter(double bytes_in, int p, const MachineSpecification& s) {
  return all_gather(bytes_in, p, s);
}
double CollectiveCost::all_to_all(double bytes, int p, const MachineSpecification& s) {
  if (p <= 1 || bytes <= 0) return 0;
  auto it = s.all_to_all_bw.find(p);
  const double bw = it != s.all_to_all_bw.end() ? it->second : eff_bw(p, s);
  return (p - 1.0) / p * bytes / bw + s.collective_latency;
}
double CollectiveCost::p2p(double bytes, const MachineSpecification& s) {
  return bytes / s.xgmi_link_bandwidth + s.collective_latency;
}

void ProfileTable::load_json(const Json& j) {
  for (auto const& kv : j.as_object()) {
    ProfileEntry e;
    e.fwd_ms = kv.second.at("fwd_ms").as_double();
    e.bwd_ms = kv.second.at("bwd_ms").as_double();
    if (kv.second.contains("resident_mb")) e.resident_mb = kv.second.at("resident_mb").as_double();
    if (kv.second.contains("peak_mb")) e.peak_mb = kv.second.at("peak_mb").as_double();
    table_[kv.first] = e;
  }
}
bool ProfileTable::lookup(const std::string& key, double& fwd, double& bwd) const {
  auto it = table_.find(key);
  if (it == table_.end()) return false;
  fwd = it->second.fwd_ms * 1e-3;
  bwd = it->second.bwd_ms * 1e-3;
  return true;
}
const ProfileEntry* ProfileTable::find(const std::string& key) const {
  auto it = table_.find(key);
  return it == table_.end() ? nullptr : &it->second;
}
void ProfileTable::put(const std::string& key, double fwd, double bwd) {
  ProfileEntry e;
  e.fwd_ms = fwd;
  e.bwd_ms = bwd;
  table_[key] = e;
}
Json ProfileTable::to_json() const {
  Json j = Json::object();
  for (auto const& kv : table_) {
    Json e = Json::object();
    e["fwd_ms"] = kv.second.fwd_ms;
    e["bwd_ms"] = kv.second.bwd_ms;
    if (kv.second.resident_mb >= 0) e["resident_mb"] = kv.second.resident_mb;
    if (kv.second.peak_mb >= 0) e["peak_mb"] = kv.second.peak_mb;
    j[kv.first] = e;
  }
  return j;
}

std::string CostModel::signature(const OpAttrs& op, const std::vector<TensorShape>& pieces) {
  std::ostringstream os;
  os << op.str();
  for (auto const& p : pieces) os << "|" << p.str();
  return os.str();
}

double CostModel::gemm_time(double flops, double bytes, double eff_hint) const {
  double eff = spec_.mfma_efficiency * std::max(0.05, std::min(1.0, eff_hint));
  return std::max(flops / (spec_.peak_bf16_flops * eff), bytes / spec_.hbm_bandwidth);
}

OpCost CostModel::op_cost(const OpAttrs& op, const std::vector<ParallelTensorShape>& inputs,
                          const std::vector<ParallelTensorShape>& weights,
                          const std::vector<ParallelTensorShape>& outputs, int block_size) const {
  size_t k = hash_combine(op.hash(), 0x0c057);
  for (auto const* v : {&inputs, &weights, &outputs}) {
    k = hash_combine(k, v->size());
    for (auto const& t : *v) k = hash_combine(k, std::hash<ParallelTensorShape>()(t));
  }
  k = hash_combine(k, static_cast<size_t>(block_size));
  {
    std::lock_guard<std::mutex> lk(memo_mu_);
    auto it = memo_.find(k);
    if (it != memo_.end()) return it->second;
  }
  OpCost c = op_cost_uncached(op, inputs, weights, outputs, block_size);
  std::lock_guard<std::mutex> lk(memo_mu_);
  memo_.emplace(k, c);
  return c;
}

OpCost CostModel::parallel_op_cost(const OpAttrs& op, const ParallelTensorShape& in, const ParallelTensorShape& out,
                                   int block_size) const {
  size_t k = hash_combine(op.hash(), 0x9a7a11e1);
  k = hash_combine(k, std::hash<ParallelTensorShape>()(in));
  k = hash_combine(k, std::hash<ParallelTensorShape>()(out));
  k = hash_combine(k, static_cast<size_t>(block_size));
  {
    std::lock_guard<std::mutex> lk(memo_mu_);
    auto it = memo_.find(k);
    if (it != memo_.end()) return it->second;
  }
  OpCost c = parallel_op_cost_uncached(op, in, out, block_size);
  std::lock_guard<std::mutex> lk(memo_mu_);
  memo_.emplace(k, c);
  return c;
}

OpCost CostModel::op_cost_uncached(const OpAttrs& op, const std::vector<ParallelTensorShape>& inputs,
                                   const std::vector<ParallelTensorShape>& weights,
                                   const std::vector<ParallelTensorShape>& outputs, int block_size) const {
  (void)block_size;
  OpCost c;
  std::vector<TensorShape> ip, wp, op_;
  for (auto const& x : inputs) ip.push_back(x.piece_shape());
  for (auto const& x : weights) wp.push_back(x.piece_shape());
  for (auto const& x : outputs) op_.push_back(x.piece_shape());
  std::vector<TensorShape> all = ip;
  all.insert(all.end(), op_.begin(), op_.end());
  const ProfileEntry* pe = profiles_.find(signature(op, all));
  if (pe) {
    c.forward = pe->fwd_ms * 1e-3;
    c.backward = pe->bwd_ms * 1e-3;
    c.measured = true;
  } else {
    // bytes at the dtype the executor computes in
    auto compute_dtype = [&](std::vector<TensorShape> v) {
      if (spec_.bf16_compute)
        for (auto& t : v)
          if (t.dtype == DataType::FLOAT) t.dtype = DataType::BFLOAT16;
      return v;
    };
    OpWork w = estimate_op_work(op, compute_dtype(ip), compute_dtype(wp), compute_dtype(op_));
    if (w.matmul_like) {
      c.forward = gemm_time(w.flops, w.bytes, w.mfma_efficiency_hint);
      c.backward = 2.0 * c.forward;
    } else {
      c.forward = std::max(w.flops / spec_.peak_fp32_flops, w.bytes / spec_.hbm_bandwidth);
      c.backward = 1.8 * c.forward;
    }
    int kernels = w.matmul_like ? 2 : 1;
    if (op.type == OpType::MULTIHEAD_ATTENTION) kernels = 4;
    if (w.flops > 0 || w.bytes > 0) {
      c.forward += kernels * spec_.kernel_launch_overhead;
      c.backward += 2 * kernels * spec_.kernel_launch_overhead;
    }
  }
  // Sequence-parallel attention (flexflow_train_amd/parallel/sequence.py):
  // the piece costs above see S/s keys, the real core attends to all S, and
  // the lowering moves data.  Ulysses (local heads divisible by s): 4
  // all-to-alls of a q-sized piece each way.  Ring: s-1 K/V block hops
  // forward (overlapped with the block compute), s hops of K/V/dK/dV back.
  if (op.type == OpType::MULTIHEAD_ATTENTION && !inputs.empty() && inputs[0].num_dims() == 3 &&
      inputs[0].dim(1).degree > 1 && !wp.empty()) {
    const int s = inputs[0].dim(1).degree;
    const double b = static_cast<double>(ip[0].dims[0]), sl = static_cast<double>(ip[0].dims[1]);
    const double h = static_cast<double>(wp[0].dims[1]);
    const double kd = op.i("kdim") > 0 ? static_cast<double>(op.i("kdim"))
                                       : static_cast<double>(op.i("embed_dim")) / static_cast<double>(op.i("num_heads"));
    double core = 4.0 * b * h * sl * sl * kd * (s - 1);
    if (op.b("causal")) core *= 0.5;
    const double core_t = gemm_time(core, 0.0, 0.8);
    const double piece = b * sl * h * kd * 2.0;  // bf16 [B, S/s, H, d]
    const bool ulysses = static_cast<int64_t>(h) % s == 0 && op.s("seq_parallel_mode") != "ring";
    if (ulysses) {
      const double a2a = CollectiveCost::all_to_all(piece, s, spec_);
      c.forward += core_t + 4 * a2a;
      c.backward += 2.5 * core_t + 4 * a2a;
    } else {
      const double hop_f = CollectiveCost::p2p(2 * piece, spec_);
      const double hop_b = CollectiveCost::p2p(2 * piece + 4 * piece, spec_);
      c.forward += std::max(core_t, (s - 1) * hop_f);
      c.backward += std::max(2.5 * core_t, s * hop_b);
    }
  }
  // Attribute (spatial) parallelism: H bands exchange halo rows with their
  // neighbours before the window op (both directions at once, one xGMI link
  // each) and return the halo gradients after its backward
  if ((op.type == OpType::CONV2D || op.type == OpType::POOL2D) && !inputs.empty() && inputs[0].num_dims() == 4 &&
      inputs[0].dim(2).degree > 1) {
    const int64_t k = op.i("kernel_h"), st = op.i("stride_h");
    const double halo_rows = static_cast<double>(std::max<int64_t>(0, k - st));
    const auto& x = ip[0];
    const double bytes = halo_rows * static_cast<double>(x.dims[0] * x.dims[1] * x.dims[3]) *
                         static_cast<double>(size_of(x.dtype));
    const double t = CollectiveCost::p2p(bytes, spec_);
    c.forward += t;
    c.backward += t;
  }
  // All-to-all expert parallelism: dispatch + combine all-to-alls forward,
  // their transposes backward (token pairs of this piece, bf16 rows).
  if (op.type == OpType::EXPERTS && op.s("expert_parallel_mode") == "alltoall" && op.i("expert_degree") > 1 &&
      ip.size() == 3) {
    const int ed = static_cast<int>(op.i("expert_degree"));
    const double pairs = static_cast<double>(ip[1].dims[0]) * static_cast<double>(ip[1].dims[1]);
    const double disp = pairs * static_cast<double>(ip[0].dims[1]) * 2.0;
    const double comb = pairs * static_cast<double>(op.i("out_dim")) * 2.0;
    const double t = CollectiveCost::all_to_all(disp, ed, spec_) + CollectiveCost::all_to_all(comb, ed, spec_);
    c.forward += t;
    c.backward += t;
  }
  // memory: weights (bf16 copy + fp32 master + fp32 m, v + grad) + saved activations
  double wmem = 0, sync = 0;
  for (size_t i = 0; i < weights.size(); ++i) {
    double elems = static_cast<double>(wp[i].num_elements());
    wmem += elems * 16.0;
    if (weights[i].discard_copy_degree > 1)
      sync += CollectiveCost::all_reduce(elems * 2.0, weights[i].discard_copy_degree, spec_);
  }
  double amem = 0;
  for (auto const& t : ip) amem += static_cast<double>(t.size_bytes());
  for (auto const& t : op_) amem += static_cast<double>(t.size_bytes());
  if (pe && pe->resident_mb >= 0) {
    // measured: what the forward leaves alive for the backward, and the
    // allocator peak over forward + backward beyond it (workspaces, input
    // gradients, recomputed intermediates)
    const double resident = pe->resident_mb * 1e6;
    amem = resident;
    if (pe->peak_mb >= 0) c.workspace = std::max(0.0, pe->peak_mb * 1e6 - resident);
  }
  c.memory = wmem + amem;
  c.sync = sync;
  return c;
}

OpCost CostModel::parallel_op_cost_uncached(const OpAttrs& op, const ParallelTensorShape& in,
                                            const ParallelTensorShape& out, int block_size) const {
  (void)block_size;
  OpCost c;
  const double in_b = static_cast<double>(in.piece_shape().size_bytes());
  const double out_b = static_cast<double>(out.piece_shape().size_bytes());
  switch (op.type) {
    case OpType::REPARTITION: {
      int d = static_cast<int>(op.i("degree"));
      c.forward = out_b / spec_.hbm_bandwidth + spec_.kernel_launch_overhead;  // local slice
      c.backward = CollectiveCost::all_gather(in_b, d, spec_);                  // gather grads
      break;
    }
    case OpType::COMBINE: {
      int d = static_cast<int>(op.i("degree"));
      c.forward = CollectiveCost::all_gather(out_b, d, spec_);
      c.backward = in_b / spec_.hbm_bandwidth + spec_.kernel_launch_overhead;
      break;
    }
    case OpType::REPLICATE: {
      int d = static_cast<int>(op.i("degree"));
      c.forward = 0;
      c.backward = op.b("partial") ? 0.0 : CollectiveCost::all_reduce(in_b, d, spec_);
      break;
    }
    case OpType::REDUCTION: {
      int d = static_cast<int>(op.i("degree"));
      c.forward = CollectiveCost::all_reduce(out_b, d, spec_);
      c.backward = 0;
      break;
    }
    case OpType::ALLTOALL: {
      int d = static_cast<int>(op.i("degree"));
      c.forward = CollectiveCost::all_to_all(in_b, d, spec_);
      c.backward = c.forward;
      break;
    }
    default:
      c.forward = c.backward = 0;
  }
  c.memory = out_b;
  return c;
}

double CostModel::movement_cost(const ParallelTensorShape& t, const Placement& src, const Placement& dst) const {
  if (src == dst || src.empty() || dst.empty()) return 0;
  const int T = std::max(1, t.total_parallel_degree());
  if (static_cast<int>(src.size()) % T || static_cast<int>(dst.size()) % T) return kMovementInfeasible;
  const int rs = static_cast<int>(src.size()) / T, rd = static_cast<int>(dst.size()) / T;
  const double piece = static_cast<double>(t.piece_shape().size_bytes());
  std::map<std::pair<int, int>, double> pair_bytes;
  std::map<int, double> in_bytes;
  for (int i = 0; i < T; ++i) {
    for (int r = 0; r < rd; ++r) {
      const int d = dst[i * rd + r];
      bool held = false;
      for (int q = 0; q < rs && !held; ++q) held = src[i * rs + q] == d;
      if (held) continue;
      const int s = src[i * rs + (r % rs)];  // spread readers over the holders
      pair_bytes[{s, d}] += piece;
      in_bytes[d] += piece;
    }
  }
  if (pair_bytes.empty()) return 0;
  const int gpn = std::max(1, spec_.num_gpus_per_node);
  double t_max = 0;
  for (auto const& kv : pair_bytes) {
    const bool inter = kv.first.first / gpn != kv.first.second / gpn;
    const double bw = inter ? spec_.inter_node_bandwidth : spec_.xgmi_link_bandwidth;
    t_max = std::max(t_max, kv.second / bw);
  }
  for (auto const& kv : in_bytes)
    t_max = std::max(t_max, kv.second / (std::max(1, spec_.xgmi_links) * spec_.xgmi_link_bandwidth));
  return t_max + spec_.collective_latency;
}

double CostModel::movement_cost(const ParallelTensorShape& t, const DeviceBlock& src, const DeviceBlock& dst) const {
  if (src == dst) return 0;
  // an unpartitioned tensor is replicated on every device of its block:
  // consumers inside that block read their local copy
  if (t.total_parallel_degree() == 1 && dst.start >= src.start && dst.start + dst.size <= src.start + src.size)
    return 0;
  return CollectiveCost::p2p(static_cast<double>(t.piece_shape().size_bytes()), spec_);
}

}  // namespace ff
