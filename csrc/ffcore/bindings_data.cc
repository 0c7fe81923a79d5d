// pybind11 bindings of the native batch prefetcher (ff/dataloader.h).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bindings_ext.h"
#include "ff/computation_graph.h"
#include "ff/dataloader.h"
#include "ff/local_exec.h"

namespace py = pybind11;

namespace ff {

namespace {
// keeps the numpy arrays alive for the prefetcher's lifetime
struct PyPrefetcher {
  std::vector<py::array> keep;
  std::unique_ptr<BatchPrefetcher> p;
};
}  // namespace

void register_data_bindings(py::module_& m) {
  py::class_<PyPrefetcher>(m, "BatchPrefetcher")
      .def(py::init([](std::vector<py::array> arrays, std::vector<std::pair<int64_t, int64_t>> rows, int64_t batch,
                       bool shuffle, uint64_t seed, int depth, int workers) {
             if (arrays.empty() || arrays.size() != rows.size())
               throw std::invalid_argument("BatchPrefetcher: one (lo, hi) row range per array");
             auto r = std::make_unique<PyPrefetcher>();
             std::vector<LoaderArray> la;
             int64_t n = -1;
             for (size_t i = 0; i < arrays.size(); ++i) {
               py::array a = arrays[i];
               if (!(a.flags() & py::array::c_style)) throw std::invalid_argument("BatchPrefetcher: arrays must be C-contiguous");
               if (a.ndim() < 1) throw std::invalid_argument("BatchPrefetcher: arrays need a sample dimension");
               const int64_t ns = a.shape(0);
               if (n >= 0 && ns != n) throw std::invalid_argument("BatchPrefetcher: arrays differ in sample count");
               n = ns;
               LoaderArray L;
               L.data = static_cast<const unsigned char*>(a.data());
               L.row_bytes = ns ? static_cast<int64_t>(a.nbytes()) / ns : 0;
               L.lo = rows[i].first;
               L.hi = rows[i].second;
               la.push_back(L);
               r->keep.push_back(a);
             }
             r->p = std::make_unique<BatchPrefetcher>(std::move(la), n, batch, shuffle, seed, depth, workers);
             return r;
           }),
           py::arg("arrays"), py::arg("rows"), py::arg("batch"), py::arg("shuffle") = false, py::arg("seed") = 0,
           py::arg("depth") = 4, py::arg("workers") = 2)
      .def("set_slot", [](PyPrefetcher& s, int slot, int a, uintptr_t ptr) {
        s.p->set_slot(slot, a, reinterpret_cast<unsigned char*>(ptr));
      })
      .def("start", [](PyPrefetcher& s, int64_t first) { s.p->start(first); }, py::arg("first_batch") = 0)
      .def("next", [](PyPrefetcher& s) {
        int64_t b = 0;
        int slot;
        {
          py::gil_scoped_release nogil;
          slot = s.p->next(&b);
        }
        return py::make_tuple(slot, b);
      })
      .def("release", [](PyPrefetcher& s, int slot) { s.p->release(slot); })
      .def("stop", [](PyPrefetcher& s) {
        py::gil_scoped_release nogil;
        s.p->stop();
      })
      .def("sample_of", [](PyPrefetcher& s, int64_t b, int64_t r) { return s.p->sample_of(b, r); })
      .def_property_readonly("iters_per_epoch", [](PyPrefetcher& s) { return s.p->iters_per_epoch(); })
      .def_property_readonly("depth", [](PyPrefetcher& s) { return s.p->depth(); });

  // ---- native CPU local execution (lib/local-execution parity)
  auto vec = [](py::array_t<float, py::array::c_style | py::array::forcecast> a) {
    return std::vector<float>(a.data(), a.data() + a.size());
  };
  py::class_<LocalTrainingBacking>(m, "LocalTrainingBacking")
      .def(py::init([](const ComputationGraph& cg, const std::string& optimizer, double lr, double momentum,
                       double weight_decay, bool nesterov, double beta1, double beta2, double epsilon,
                       const std::string& loss, uint64_t seed) {
             LocalOptimizer o;
             o.kind = optimizer;
             o.lr = lr;
             o.momentum = momentum;
             o.weight_decay = weight_decay;
             o.nesterov = nesterov;
             o.beta1 = beta1;
             o.beta2 = beta2;
             o.epsilon = epsilon;
             return std::make_unique<LocalTrainingBacking>(cg, o, loss, seed);
           }),
           py::arg("cg"), py::arg("optimizer") = "sgd", py::arg("lr") = 0.01, py::arg("momentum") = 0.0,
           py::arg("weight_decay") = 0.0, py::arg("nesterov") = false, py::arg("beta1") = 0.9,
           py::arg("beta2") = 0.999, py::arg("epsilon") = 1e-8,
           py::arg("loss") = "sparse_categorical_crossentropy", py::arg("seed") = 0, py::keep_alive<1, 2>())
      .def("input_names", &LocalTrainingBacking::input_names)
      .def("weight_names", &LocalTrainingBacking::weight_names)
      .def("shape_of", &LocalTrainingBacking::shape_of)
      .def("set_input", [=](LocalTrainingBacking& b, const std::string& n,
                            py::array_t<float, py::array::c_style | py::array::forcecast> a) {
        b.set_input(n, vec(a));
      })
      .def("set_weight", [=](LocalTrainingBacking& b, const std::string& n,
                             py::array_t<float, py::array::c_style | py::array::forcecast> a) {
        b.set_weight(n, vec(a));
      })
      .def("get_weight", [](const LocalTrainingBacking& b, const std::string& n) {
        auto v = b.get_weight(n);
        auto shp = b.shape_of(n);
        py::array_t<float> r(shp);
        std::copy(v.begin(), v.end(), r.mutable_data());
        return r;
      })
      .def("get_output", [](const LocalTrainingBacking& b) {
        auto v = b.get_output();
        py::array_t<float> r(static_cast<py::ssize_t>(v.size()));
        std::copy(v.begin(), v.end(), r.mutable_data());
        return r;
      })
      .def("forward", [](LocalTrainingBacking& b) {
        py::gil_scoped_release nogil;
        b.forward();
      })
      .def("backward", [=](LocalTrainingBacking& b, py::array_t<float, py::array::c_style | py::array::forcecast> y) {
        auto v = vec(y);
        py::gil_scoped_release nogil;
        b.backward(v);
      })
      .def("update", [](LocalTrainingBacking& b) {
        py::gil_scoped_release nogil;
        b.update();
      })
      .def("train_step", [=](LocalTrainingBacking& b, py::array_t<float, py::array::c_style | py::array::forcecast> y) {
        auto v = vec(y);
        py::gil_scoped_release nogil;
        b.train_step(v);
      })
      .def("metrics", [](const LocalTrainingBacking& b) {
        const auto& m = b.metrics();
        py::dict d;
        d["loss_sum"] = m.loss_sum;
        d["correct"] = m.correct;
        d["samples"] = m.samples;
        return d;
      })
      .def("reset_metrics", &LocalTrainingBacking::reset_metrics)
      .def("layer_times_ms", &LocalTrainingBacking::layer_times_ms)
      .def_static("registered_ops", [] {
        std::vector<std::string> r;
        for (auto const& kv : LocalTrainingBacking::registry()) r.push_back(to_string(kv.first));
        return r;
      });
  m.def("measure_op_cost_ms", [](const OpAttrs& op, const std::vector<TensorShape>& shapes, int iters) {
    return measure_op_cost_ms(op, shapes, iters);
  }, py::arg("op"), py::arg("input_shapes"), py::arg("iters") = 3);
}

}  // namespace ff
