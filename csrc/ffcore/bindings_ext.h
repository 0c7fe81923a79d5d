// Hook for bindings of the search/simulator subsystems (bindings_search.cc).
#pragma once
#include <pybind11/pybind11.h>

#include "ff/op_attrs.h"

namespace ff {
void register_ext_bindings(pybind11::module_& m);
void register_data_bindings(pybind11::module_& m);
AttrValue py_to_attr(const pybind11::handle& o);
pybind11::object attr_to_py(const AttrValue& v);
}  // namespace ff
