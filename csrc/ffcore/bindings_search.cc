// Bindings for machine mapping / search / simulator (filled in as those land).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bindings_ext.h"

namespace py = pybind11;

namespace ff {
void register_ext_bindings(py::module_& m) { (void)m; }
}  // namespace ff
