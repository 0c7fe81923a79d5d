// Topology-aware network model: devices + switches joined by links, routes,
// and collectives priced by the load they put on every link.
//
// Parity: the reference's NetworkedMachineModel / EnhancedMachineModel
// (lib/runtime/src/machine_model.cc:58-146, 966-1287), its routing strategies
// (WeightedShortestPathRoutingStrategy, ShortestPathNetworkRoutingStrategy
// with ECMP, network.cc:47-587), topology generators (FlatDegConstraint,
// BigSwitch, FullyConnected, simulator.h:330-455) and the ring expansion of
// all-reduce over routed links (LogicalTaskgraphBasedSimulator::
// expand_allreduce, simulator.cc:1684-1795), plus the machine config file
// format (machine_config_example:1-60).
//
// MI355X-first: a node is 8 GPUs fully connected by xGMI (one link per GPU
// pair, 7 per GPU); RCCL runs several rings over disjoint links at once, so
// an all-reduce is modelled as `R` concurrent rings (strides coprime with p)
// splitting the data, and its time is the most loaded link's bytes over its
// bandwidth plus per-step latency.  Nodes are joined through per-GPU NICs to
// a switch.  The model yields effective collective bandwidths per group size
// that the analytic cost model (machine.h) then uses.
#pragma once
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "ff/json.h"
#include "ff/machine.h"

namespace ff {

struct NetLink {
  int u = 0, v = 0;          // directed u -> v
  double bandwidth = 0;      // bytes / s
  double latency = 0;        // s
};

class NetworkTopology {
 public:
  // GPUs are vertices [0, num_devices); switches / NICs follow.
  int num_devices = 0;
  int num_vertices = 0;
  std::vector<NetLink> links;
  std::string name;

  void add_bidirectional(int a, int b, double bw, double lat);
  int add_vertex();
  // adjacency: vertex -> list of link indices leaving it
  std::vector<std::vector<int>> adjacency() const;

  // ---- generators
  static NetworkTopology fully_connected(int n, double link_bw, double latency);
  static NetworkTopology big_switch(int n, double link_bw, double latency);
  // random `degree`-regular-ish graph (FlatDegConstraint), deterministic in `seed`
  static NetworkTopology flat_deg_constraint(int n, int degree, double link_bw, double latency, uint64_t seed);
  // `nodes` MI355X nodes: xGMI mesh inside, one NIC per GPU into a switch
  static NetworkTopology mi355x_cluster(int nodes, int gpus_per_node, double xgmi_bw, double xgmi_lat,
                                        double nic_bw, double nic_lat);
  // "key = value" machine config (reference machine_config_example keys plus
  // xgmi_*, nic_*, topology = mi355x | fully_connected | big_switch | flat_deg)
  static NetworkTopology from_config_text(const std::string& text, MachineSpecification* spec_out = nullptr);
  static NetworkTopology from_config_file(const std::string& path, MachineSpecification* spec_out = nullptr);
  Json to_json() const;
};

enum class RoutingStrategy { WEIGHTED_SHORTEST_PATH = 0, SHORTEST_PATH_ECMP = 1 };

class NetworkModel {
 public:
  NetworkModel(NetworkTopology t, RoutingStrategy r = RoutingStrategy::SHORTEST_PATH_ECMP, int max_rings = 4);
  const NetworkTopology& topology() const { return topo_; }

  // routes src -> dst: a set of paths (link index lists) sharing the traffic
  const std::vector<std::vector<int>>& routes(int src, int dst) const;
  double p2p_time(int src, int dst, double bytes) const;
  // collectives over an ordered device group
  double all_reduce_time(const std::vector<int>& devs, double bytes) const;
  double all_gather_time(const std::vector<int>& devs, double bytes_out) const;
  double all_to_all_time(const std::vector<int>& devs, double bytes) const;
  // effective bus bandwidths (bytes/s) of consecutive blocks of p devices,
  // written into spec.collective_bw / spec.all_to_all_bw
  void calibrate(MachineSpecification& spec, double probe_bytes = 256.0 * (1 << 20)) const;

 private:
  NetworkTopology topo_;
  RoutingStrategy strategy_;
  int max_rings_;
  mutable std::map<std::pair<int, int>, std::vector<std::vector<int>>> cache_;
  std::vector<std::vector<int>> compute_routes(int src, int dst) const;
  double max_load_time(const std::map<int, double>& link_bytes) const;
  double path_latency(const std::vector<int>& path) const;
};

}  // namespace ff
