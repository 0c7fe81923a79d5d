// pybind11 bindings of the native batch prefetcher (ff/dataloader.h).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bindings_ext.h"
#include "ff/dataloader.h"

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
}

}  // namespace ff
