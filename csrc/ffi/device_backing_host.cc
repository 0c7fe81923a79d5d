// Host-only definition of ff::make_device_backing for builds that compile no
// HIP code (the host-code sanitizer build, tools/build_native.py "asan"): the
// C runtime API then always trains on the CPU backing.  The GPU definition is
// csrc/ffdev/device_exec.cpp, linked into libflexflow_runtime_c.so.
#include "ff/training_backing.h"

namespace ff {

std::unique_ptr<TrainingBacking> make_device_backing(const ComputationGraph&, LocalOptimizer, const std::string&,
                                                     uint64_t, std::string* why) {
  if (why) *why = "host-only build (no HIP device code linked)";
  return nullptr;
}

}  // namespace ff
