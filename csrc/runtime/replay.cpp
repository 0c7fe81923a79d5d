// Native replay of a segmented distributed training step (the thin host
// executor of SURVEY §7.1 for multi-GPU runs).
//
// runtime/graphs.py captures a distributed step as a chain of hipGraph
// SEGMENTS cut at every collective.  The Python replay walked that chain in
// the interpreter: one graph launch, then the collective re-issued through
// torch.distributed, then the next launch ... -- the interpreter sat on the
// critical path between segments (25 segments / 13 collectives per BERT step
// in the round-4 rehearsal).  This replayer holds the chain as C++ items and
// walks it in one call: graph launches go straight to at::cuda::CUDAGraph,
// collectives straight to the c10d::ProcessGroup (RCCL on ROCm) with the
// same options torch.distributed would pass, and async works are waited on
// at the recorded points.  Stream semantics are torch.distributed's: each
// collective is enqueued behind the current stream's work (the segment just
// launched) and the next segment runs while it reduces.
//
// Parity: the reference replays Legion traces around each iteration
// (python/flexflow/core/flexflow_cffi.py:562-566, begin_trace / end_trace)
// and issues its NCCL collectives from C++ tasks
// (lib/runtime/src/optimizer_kernel.cu NCCL update).
#include <torch/extension.h>

#include <ATen/hip/HIPGraph.h>   // at::cuda::CUDAGraph on ROCm builds of torch
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

enum Kind : int {
  kGraph = 0,
  kAllReduce = 1,
  kReduceScatter = 2,   // out = chunk of in (reduce_scatter_tensor)
  kAllGather = 3,       // out = gathered in (all_gather_into_tensor)
  kReduce = 4,
  kBroadcast = 5,
  kWait = 6,
  kAllToAll = 7,        // out = all_to_all_single(in, out / in split sizes)
  kSendRecv = 8,        // matched point-to-point pairs (a pipeline-stage boundary), one coalesced group
};

struct Item {
  int kind = kGraph;
  py::object graph;   // keeps the Python CUDAGraph (and its pool) alive
  at::cuda::CUDAGraph* g = nullptr;
  c10::intrusive_ptr<c10d::ProcessGroup> pg;
  at::Tensor a, b;    // collective operands (in / out)
  int root = 0;       // group-local root rank (reduce / broadcast)
  int slot = -1;      // async work slot (-1: synchronous), or the slot waited on
  std::vector<int64_t> out_splits, in_splits;   // all-to-all (empty: equal splits)
  std::vector<int> send_peers, recv_peers;      // send / recv: group ranks
  std::vector<at::Tensor> sends, recvs;
};

class Replayer {
 public:
  void add_graph(py::object graph) {
    Item it;
    it.kind = kGraph;
    it.g = graph.cast<at::cuda::CUDAGraph*>();
    it.graph = std::move(graph);
    items_.push_back(std::move(it));
  }
  void add_collective(int kind, const c10::intrusive_ptr<c10d::ProcessGroup>& pg, at::Tensor a, at::Tensor b,
                      int root, int slot, std::vector<int64_t> out_splits, std::vector<int64_t> in_splits) {
    if (kind < kAllReduce || kind > kAllToAll || kind == kWait)
      throw std::invalid_argument("replay: unknown collective kind");
    if (!pg) throw std::invalid_argument("replay: null process group");
    Item it;
    it.kind = kind;
    it.pg = pg;
    it.a = std::move(a);
    it.b = std::move(b);
    it.root = root;
    it.slot = slot;
    it.out_splits = std::move(out_splits);
    it.in_splits = std::move(in_splits);
    items_.push_back(std::move(it));
  }
  void add_send_recv(const c10::intrusive_ptr<c10d::ProcessGroup>& pg, std::vector<int> send_peers,
                     std::vector<at::Tensor> sends, std::vector<int> recv_peers, std::vector<at::Tensor> recvs,
                     int slot) {
    if (!pg) throw std::invalid_argument("replay: null process group");
    if (send_peers.size() != sends.size() || recv_peers.size() != recvs.size() || (sends.empty() && recvs.empty()))
      throw std::invalid_argument("replay: send / recv lists do not match");
    Item it;
    it.kind = kSendRecv;
    it.pg = pg;
    it.send_peers = std::move(send_peers);
    it.sends = std::move(sends);
    it.recv_peers = std::move(recv_peers);
    it.recvs = std::move(recvs);
    it.slot = slot;
    items_.push_back(std::move(it));
  }
  void add_wait(int slot) {
    Item it;
    it.kind = kWait;
    it.slot = slot;
    items_.push_back(std::move(it));
  }
  size_t size() const { return items_.size(); }
  int n_graphs() const {
    int n = 0;
    for (const auto& it : items_) n += it.kind == kGraph;
    return n;
  }

  void replay() {
    std::map<int, c10::intrusive_ptr<c10d::Work>> works;
    {
      py::gil_scoped_release nogil;   // the whole step runs without the interpreter
      for (auto& it : items_) {
        switch (it.kind) {
          case kGraph: it.g->replay(); break;
          case kWait: {
            auto w = works.find(it.slot);
            if (w != works.end()) {
              w->second->wait();
              works.erase(w);
            }
            break;
          }
          default: {
            auto w = issue(it);
            if (it.slot >= 0) works[it.slot] = w;
            else w->wait();   // synchronous semantics: the stream waits (as dist.* with async_op=False)
          }
        }
      }
      for (auto& kv : works) kv.second->wait();   // never waited inside the step: keep stream order
    }
  }

 private:
  static c10::intrusive_ptr<c10d::Work> issue(Item& it) {
    if (it.kind == kSendRecv) {
      // RCCL: one coalesced group (ncclGroupStart / End), as
      // torch.distributed.batch_isend_irecv issues it; other backends (gloo
      // rehearsals) post every op and wait them all
      const bool cuda = !it.sends.empty() ? it.sends[0].is_cuda() : (!it.recvs.empty() && it.recvs[0].is_cuda());
      const bool coalesce = cuda && it.pg->getBackendName() == "nccl";
      if (coalesce) it.pg->startCoalescing(c10::DeviceType::CUDA);
      std::vector<c10::intrusive_ptr<c10d::Work>> ws;
      for (size_t i = 0; i < it.sends.size(); ++i) {
        std::vector<at::Tensor> v{it.sends[i]};
        ws.push_back(it.pg->send(v, it.send_peers[i], 0));
      }
      for (size_t i = 0; i < it.recvs.size(); ++i) {
        std::vector<at::Tensor> v{it.recvs[i]};
        ws.push_back(it.pg->recv(v, it.recv_peers[i], 0));
      }
      if (coalesce) return it.pg->endCoalescing(c10::DeviceType::CUDA);
      for (size_t i = 0; i + 1 < ws.size(); ++i) ws[i]->wait();
      return ws.back();
    }
    switch (it.kind) {
      case kAllReduce: {
        std::vector<at::Tensor> v{it.a};
        c10d::AllreduceOptions o;
        o.reduceOp = c10d::ReduceOp::SUM;
        return it.pg->allreduce(v, o);
      }
      case kReduceScatter: {
        c10d::ReduceScatterOptions o;
        o.reduceOp = c10d::ReduceOp::SUM;
        return it.pg->_reduce_scatter_base(it.b, it.a, o);
      }
      case kAllGather: {
        c10d::AllgatherOptions o;
        return it.pg->_allgather_base(it.b, it.a, o);
      }
      case kReduce: {
        std::vector<at::Tensor> v{it.a};
        c10d::ReduceOptions o;
        o.reduceOp = c10d::ReduceOp::SUM;
        o.rootRank = it.root;
        return it.pg->reduce(v, o);
      }
      case kBroadcast: {
        std::vector<at::Tensor> v{it.a};
        c10d::BroadcastOptions o;
        o.rootRank = it.root;
        return it.pg->broadcast(v, o);
      }
      case kAllToAll: {
        c10d::AllToAllOptions o;
        return it.pg->alltoall_base(it.b, it.a, it.out_splits, it.in_splits, o);
      }
      default: throw std::invalid_argument("replay: not a collective");
    }
  }

  std::vector<Item> items_;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "native replay of segmented distributed hipGraph steps (graphs + RCCL collectives)";
  py::class_<Replayer>(m, "Replayer")
      .def(py::init<>())
      .def("add_graph", &Replayer::add_graph)
      .def("add_collective", &Replayer::add_collective, py::arg("kind"), py::arg("pg"), py::arg("a"), py::arg("b"),
           py::arg("root"), py::arg("slot"), py::arg("out_splits") = std::vector<int64_t>{},
           py::arg("in_splits") = std::vector<int64_t>{})
      .def("add_send_recv", &Replayer::add_send_recv, py::arg("pg"), py::arg("send_peers"), py::arg("sends"),
           py::arg("recv_peers"), py::arg("recvs"), py::arg("slot"))
      .def("add_wait", &Replayer::add_wait)
      .def("replay", &Replayer::replay)
      .def("__len__", &Replayer::size)
      .def("n_graphs", &Replayer::n_graphs);
  m.attr("ALL_REDUCE") = static_cast<int>(kAllReduce);
  m.attr("REDUCE_SCATTER") = static_cast<int>(kReduceScatter);
  m.attr("ALL_GATHER") = static_cast<int>(kAllGather);
  m.attr("REDUCE") = static_cast<int>(kReduce);
  m.attr("BROADCAST") = static_cast<int>(kBroadcast);
  m.attr("ALL_TO_ALL") = static_cast<int>(kAllToAll);
  m.attr("SEND_RECV") = static_cast<int>(kSendRecv);
}
