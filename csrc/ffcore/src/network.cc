#include "ff/network.h"

#include <algorithm>
#include <cmath>
#include <fstream>
#include <functional>
#include <limits>
#include <numeric>
#include <queue>
#include <random>
#include <set>
#include <sstream>

namespace ff {

// ------------------------------------------------------------- topology
int NetworkTopology::add_vertex() { return num_vertices++; }

void NetworkTopology::add_bidirectional(int a, int b, double bw, double lat) {
  links.push_back({a, b, bw, lat});
  links.push_back({b, a, bw, lat});
}

std::vector<std::vector<int>> NetworkTopology::adjacency() const {
  std::vector<std::vector<int>> adj(num_vertices);
  for (size_t i = 0; i < links.size(); ++i) adj[links[i].u].push_back(static_cast<int>(i));
  return adj;
}

NetworkTopology NetworkTopology::fully_connected(int n, double bw, double lat) {
  NetworkTopology t;
  t.name = "fully_connected";
  t.num_devices = t.num_vertices = n;
  for (int a = 0; a < n; ++a)
    for (int b = a + 1; b < n; ++b) t.add_bidirectional(a, b, bw, lat);
  return t;
}

NetworkTopology NetworkTopology::big_switch(int n, double bw, double lat) {
  NetworkTopology t;
  t.name = "big_switch";
  t.num_devices = t.num_vertices = n;
  const int sw = t.add_vertex();
  for (int a = 0; a < n; ++a) t.add_bidirectional(a, sw, bw, lat / 2);
  return t;
}

NetworkTopology NetworkTopology::flat_deg_constraint(int n, int degree, double bw, double lat, uint64_t seed) {
  NetworkTopology t;
  t.name = "flat_deg_constraint";
  t.num_devices = t.num_vertices = n;
  std::mt19937_64 rng(seed);
  std::vector<int> deg(n, 0);
  std::set<std::pair<int, int>> edges;
  // a ring first keeps the graph connected, then random chords up to `degree`
  for (int a = 0; a < n && n > 1; ++a) {
    int b = (a + 1) % n;
    auto e = std::minmax(a, b);
    if (edges.insert({e.first, e.second}).second) {
      ++deg[a];
      ++deg[b];
    }
  }
  for (int tries = 0; tries < n * degree * 20; ++tries) {
    int a = static_cast<int>(rng() % n), b = static_cast<int>(rng() % n);
    if (a == b || deg[a] >= degree || deg[b] >= degree) continue;
    auto e = std::minmax(a, b);
    if (edges.insert({e.first, e.second}).second) {
      ++deg[a];
      ++deg[b];
    }
  }
  for (auto const& e : edges) t.add_bidirectional(e.first, e.second, bw, lat);
  return t;
}

NetworkTopology NetworkTopology::mi355x_cluster(int nodes, int g, double xgmi_bw, double xgmi_lat, double nic_bw,
                                                double nic_lat) {
  NetworkTopology t;
  t.name = "mi355x_cluster";
  t.num_devices = t.num_vertices = nodes * g;
  for (int n = 0; n < nodes; ++n)
    for (int a = 0; a < g; ++a)
      for (int b = a + 1; b < g; ++b) t.add_bidirectional(n * g + a, n * g + b, xgmi_bw, xgmi_lat);
  if (nodes > 1) {
    const int sw = t.add_vertex();
    for (int d = 0; d < nodes * g; ++d) t.add_bidirectional(d, sw, nic_bw, nic_lat / 2);
  }
  return t;
}

NetworkTopology NetworkTopology::from_config_text(const std::string& text, MachineSpecification* spec_out) {
  std::map<std::string, std::string> kv;
  std::istringstream in(text);
  std::string line;
  while (std::getline(in, line)) {
    auto h = line.find('#');
    if (h != std::string::npos) line = line.substr(0, h);
    auto eq = line.find('=');
    if (eq == std::string::npos) continue;
    auto trim = [](std::string s) {
      s.erase(0, s.find_first_not_of(" \t\r"));
      s.erase(s.find_last_not_of(" \t\r") + 1);
      return s;
    };
    kv[trim(line.substr(0, eq))] = trim(line.substr(eq + 1));
  }
  auto num = [&](const char* k, double d) { return kv.count(k) ? std::stod(kv[k]) : d; };
  const int nodes = static_cast<int>(num("num_nodes", 1));
  // GPUs per node: ours, or the reference's sockets x gpus_per_socket
  int g = static_cast<int>(num("num_gpus_per_node", 0));
  if (g <= 0) g = static_cast<int>(num("num_sockets_per_node", 1) * num("num_gpus_per_socket", 8));
  // bandwidths are GB/s and latencies ms in the reference format
  const double xbw = num("xgmi_bandwidth", num("nvlink_bandwidth", 64.0)) * 1e9;
  const double xlat = num("xgmi_latency", num("nvlink_latency", 0.001)) * 1e-3;
  const double nbw = num("nic_bandwidth", 50.0) * 1e9;
  const double nlat = num("nic_latency", 0.005) * 1e-3;
  std::string topo = kv.count("topology") ? kv["topology"] : "mi355x";
  NetworkTopology t;
  if (topo == "fully_connected") t = fully_connected(nodes * g, xbw, xlat);
  else if (topo == "big_switch") t = big_switch(nodes * g, xbw, xlat);
  else if (topo == "flat_deg" || topo == "flat_deg_constraint")
    t = flat_deg_constraint(nodes * g, static_cast<int>(num("degree", 4)), xbw, xlat,
                            static_cast<uint64_t>(num("seed", 1)));
  else t = mi355x_cluster(nodes, g, xbw, xlat, nbw, nlat);
  if (spec_out) {
    spec_out->num_nodes = nodes;
    spec_out->num_gpus_per_node = g;
    spec_out->xgmi_link_bandwidth = xbw;
    spec_out->inter_node_bandwidth = nbw;
    spec_out->num_cpus_per_node = static_cast<int>(num("num_sockets_per_node", 1) * num("num_cpus_per_socket", 1));
  }
  return t;
}

NetworkTopology NetworkTopology::from_config_file(const std::string& path, MachineSpecification* spec_out) {
  std::ifstream f(path);
  if (!f) throw FFError("cannot read machine config " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return from_config_text(ss.str(), spec_out);
}

Json NetworkTopology::to_json() const {
  Json j = Json::object();
  j["name"] = name;
  j["num_devices"] = num_devices;
  j["num_vertices"] = num_vertices;
  Json ls = Json::array();
  for (auto const& l : links) {
    Json e = Json::object();
    e["u"] = l.u;
    e["v"] = l.v;
    e["bandwidth"] = l.bandwidth;
    e["latency"] = l.latency;
    ls.push_back(e);
  }
  j["links"] = ls;
  return j;
}

// ---------------------------------------------------------------- model
NetworkModel::NetworkModel(NetworkTopology t, RoutingStrategy r, int max_rings)
    : topo_(std::move(t)), strategy_(r), max_rings_(std::max(1, max_rings)) {}

double NetworkModel::path_latency(const std::vector<int>& path) const {
  double l = 0;
  for (int e : path) l += topo_.links[e].latency;
  return l;
}

std::vector<std::vector<int>> NetworkModel::compute_routes(int src, int dst) const {
  if (src == dst) return {{}};
  auto adj = topo_.adjacency();
  const int V = topo_.num_vertices;
  // edge cost: hops (ECMP) or latency + 1 GB transfer time (weighted)
  auto cost = [&](int e) {
    if (strategy_ == RoutingStrategy::SHORTEST_PATH_ECMP) return 1.0;
    return topo_.links[e].latency + 1e9 / topo_.links[e].bandwidth;
  };
  std::vector<double> dist(V, std::numeric_limits<double>::infinity());
  std::vector<std::vector<int>> pred(V);  // incoming link indices on shortest paths
  using Q = std::pair<double, int>;
  std::priority_queue<Q, std::vector<Q>, std::greater<Q>> pq;
  dist[src] = 0;
  pq.push({0, src});
  while (!pq.empty()) {
    auto [d, u] = pq.top();
    pq.pop();
    if (d > dist[u] + 1e-12) continue;
    for (int e : adj[u]) {
      const int v = topo_.links[e].v;
      // switches / NICs relay; devices other than src/dst do not forward
      if (v != dst && v < topo_.num_devices) {
        // GPU-to-GPU forwarding is allowed only on device-only topologies
        bool has_switch = topo_.num_vertices > topo_.num_devices;
        if (has_switch) continue;
      }
      const double nd = d + cost(e);
      if (nd < dist[v] - 1e-12) {
        dist[v] = nd;
        pred[v] = {e};
        pq.push({nd, v});
      } else if (std::fabs(nd - dist[v]) <= 1e-12) {
        pred[v].push_back(e);
      }
    }
  }
  if (!std::isfinite(dist[dst])) throw FFError("network: no route between devices");
  // enumerate shortest paths back from dst (ECMP keeps up to 8)
  std::vector<std::vector<int>> out;
  std::vector<int> cur;
  std::function<void(int)> rec = [&](int v) {
    if (out.size() >= (strategy_ == RoutingStrategy::SHORTEST_PATH_ECMP ? 8u : 1u)) return;
    if (v == src) {
      out.emplace_back(cur.rbegin(), cur.rend());
      return;
    }
    for (int e : pred[v]) {
      cur.push_back(e);
      rec(topo_.links[e].u);
      cur.pop_back();
    }
  };
  rec(dst);
  return out;
}

const std::vector<std::vector<int>>& NetworkModel::routes(int src, int dst) const {
  auto key = std::make_pair(src, dst);
  auto it = cache_.find(key);
  if (it != cache_.end()) return it->second;
  return cache_[key] = compute_routes(src, dst);
}

double NetworkModel::max_load_time(const std::map<int, double>& link_bytes) const {
  double t = 0;
  for (auto const& kv : link_bytes) t = std::max(t, kv.second / topo_.links[kv.first].bandwidth);
  return t;
}

static void add_flow(const NetworkModel& m, std::map<int, double>& load, int s, int d, double bytes) {
  auto const& rs = m.routes(s, d);
  const double share = bytes / static_cast<double>(rs.size());
  for (auto const& p : rs)
    for (int e : p) load[e] += share;
}

double NetworkModel::p2p_time(int src, int dst, double bytes) const {
  if (src == dst || bytes <= 0) return 0;
  std::map<int, double> load;
  add_flow(*this, load, src, dst, bytes);
  return max_load_time(load) + path_latency(routes(src, dst)[0]);
}

double NetworkModel::all_reduce_time(const std::vector<int>& devs, double bytes) const {
  const int p = static_cast<int>(devs.size());
  if (p <= 1 || bytes <= 0) return 0;
  // rings i -> i + s (mod p) for strides coprime with p; data split evenly
  std::vector<int> strides;
  for (int s = 1; s < p && static_cast<int>(strides.size()) < max_rings_; ++s)
    if (std::gcd(s, p) == 1) strides.push_back(s);
  const double per_ring = bytes / static_cast<double>(strides.size());
  std::map<int, double> load;
  double lat = 0;
  for (int s : strides) {
    // reduce-scatter + all-gather: every ring hop carries 2 (p-1)/p of the ring's share
    for (int i = 0; i < p; ++i) add_flow(*this, load, devs[i], devs[(i + s) % p], 2.0 * (p - 1) / p * per_ring);
    lat = std::max(lat, path_latency(routes(devs[0], devs[s % p])[0]));
  }
  return max_load_time(load) + 2.0 * (p - 1) * lat;
}

double NetworkModel::all_gather_time(const std::vector<int>& devs, double bytes_out) const {
  const int p = static_cast<int>(devs.size());
  if (p <= 1 || bytes_out <= 0) return 0;
  return 0.5 * all_reduce_time(devs, bytes_out);
}

double NetworkModel::all_to_all_time(const std::vector<int>& devs, double bytes) const {
  const int p = static_cast<int>(devs.size());
  if (p <= 1 || bytes <= 0) return 0;
  std::map<int, double> load;
  double lat = 0;
  for (int a = 0; a < p; ++a)
    for (int b = 0; b < p; ++b)
      if (a != b) {
        add_flow(*this, load, devs[a], devs[b], bytes / p);
        lat = std::max(lat, path_latency(routes(devs[a], devs[b])[0]));
      }
  return max_load_time(load) + lat;
}

void NetworkModel::calibrate(MachineSpecification& spec, double probe) const {
  for (int p = 2; p <= topo_.num_devices; p *= 2) {
    std::vector<int> devs(p);
    std::iota(devs.begin(), devs.end(), 0);
    const double ar = all_reduce_time(devs, probe);
    spec.collective_bw[p] = 2.0 * (p - 1) / p * probe / std::max(ar, 1e-12);
    const double a2a = all_to_all_time(devs, probe);
    spec.all_to_all_bw[p] = (p - 1.0) / p * probe / std::max(a2a, 1e-12);
  }
}

}  // namespace ff
