#!/usr/bin/env python3
"""Build the native parts of flexflow_train_amd in-tree.

Two shared objects are produced next to the Python package:

* ``_ffcore``    - the C++17 core (IR, shape inference, PCG, substitutions,
                   machine mapping, Unity/MCMC search, simulator), g++ + pybind11.
* ``_ffkernels`` - hand-written HIP kernels for gfx950 (CDNA4), hipcc + pybind11.

A ``build.ninja`` is generated under ``build/`` so rebuilds are incremental and
header dependencies are tracked through compiler depfiles.  Usage::

    python tools/build_native.py            # build both
    python tools/build_native.py core       # only _ffcore
    python tools/build_native.py kernels    # only _ffkernels
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "build")
PKG = os.path.join(ROOT, "flexflow_train_amd")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("FF_OFFLOAD_ARCH", "gfx950")


def _pybind_includes() -> list[str]:
    import pybind11

    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _rel(p: str) -> str:
    return os.path.relpath(p, BUILD)


def write_ninja(targets: list[str]) -> str:
    inc = " ".join(f"-I{p}" for p in _pybind_includes())
    core_inc = f"-I{os.path.join(ROOT, 'csrc', 'ffcore', 'include')}"
    kern_inc = f"-I{os.path.join(ROOT, 'csrc', 'kernels')}"
    cxx = os.environ.get("CXX", "g++")
    lines = [
        "ninja_required_version = 1.5",
        f"cxx = {cxx}",
        f"hipcc = {HIPCC}",
        f"core_flags = -O2 -g0 -std=c++17 -fPIC -fvisibility=hidden -Wall -Wno-unused-function {core_inc} "
        f"-I{os.path.join(ROOT, 'csrc', 'ffi')} {inc}",
        # -mcode-object-version=5 keeps the code object loadable by the HIP
        # runtime bundled with the PyTorch wheel (ROCm 7.0) as well as 7.2.
        f"hip_flags = -O3 -std=c++17 -fPIC --offload-arch={ARCH} -mcode-object-version=5 "
        f"-fvisibility=hidden -munsafe-fp-atomics -Wno-unused-result {kern_inc} {inc}",
        "rule cxx",
        "  command = $cxx $core_flags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX $in",
        "rule hip",
        "  command = $hipcc $hip_flags -MMD -MF $out.d -c $in -o $out",
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule link_cxx",
        "  command = $cxx -shared -o $out $in -lpthread",
        "  description = LINK $out",
        "rule link_hip",
        f"  command = $hipcc -shared --offload-arch={ARCH} -o $out $in -L{os.path.join(ROCM, 'lib')} -lhipblaslt",
        "  description = LINK $out",
    ]
    defaults = []
    if "core" in targets:
        srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "ffcore", "src", "*.cc")))
        srcs += sorted(glob.glob(os.path.join(ROOT, "csrc", "ffcore", "bindings*.cc")))
        objs = []
        for s in srcs:
            o = os.path.join("obj", "core", os.path.basename(s) + ".o")
            lines.append(f"build {o}: cxx {s}")
            objs.append(o)
        out = os.path.join(PKG, "_ffcore" + EXT)
        lines.append(f"build {out}: link_cxx {' '.join(objs)}")
        defaults.append(out)
    if "kernels" in targets:
        srcs = sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip")))
        srcs += sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "bindings*.cpp")))
        objs = []
        for s in srcs:
            o = os.path.join("obj", "kernels", os.path.basename(s) + ".o")
            lines.append(f"build {o}: hip {s}")
            objs.append(o)
        out = os.path.join(PKG, "_ffkernels" + EXT)
        lines.append(f"build {out}: link_hip {' '.join(objs)}")
        defaults.append(out)
    if "tools" in targets:
        # native CLIs (bin/): export-model-arch, substitution-to-dot, protobuf-to-json
        lines += ["rule link_exe", "  command = $cxx -o $out $in -lpthread", "  description = LINK $out"]
        core_objs = []
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "ffcore", "src", "*.cc"))):
            o = os.path.join("obj", "core", os.path.basename(s) + ".o")
            if "core" not in targets:
                lines.append(f"build {o}: cxx {s}")
            core_objs.append(o)
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "tools", "*.cc"))):
            o = os.path.join("obj", "tools", os.path.basename(s) + ".o")
            lines.append(f"build {o}: cxx {s}")
            exe = os.path.join(ROOT, "bin", "ffc-" + os.path.basename(s)[:-3].replace("_", "-"))
            lines.append(f"build {exe}: link_exe {o} {' '.join(core_objs)}")
            defaults.append(exe)
    if "ffi" in targets:
        # C ABI (csrc/ffi/flexflow_c.h): libflexflow_c.so + a C smoke program
        lines += ["rule link_so", "  command = $cxx -shared -o $out $in -lpthread", "  description = LINK $out",
                  "rule cc_exe",
                  f"  command = gcc -O2 -std=c11 -I{os.path.join(ROOT, 'csrc', 'ffi')} -o $out $in "
                  f"-L{os.path.join(PKG, 'lib')} -lflexflow_c -Wl,-rpath,{os.path.join(PKG, 'lib')}",
                  "  description = CC $out"]
        core_objs = []
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "ffcore", "src", "*.cc"))):
            o = os.path.join("obj", "core", os.path.basename(s) + ".o")
            if "core" not in targets and "tools" not in targets:
                lines.append(f"build {o}: cxx {s}")
            core_objs.append(o)
        fo = os.path.join("obj", "ffi", "flexflow_c.cc.o")
        lines.append(f"build {fo}: cxx {os.path.join(ROOT, 'csrc', 'ffi', 'flexflow_c.cc')}")
        lib = os.path.join(PKG, "lib", "libflexflow_c.so")
        lines.append(f"build {lib}: link_so {fo} {' '.join(core_objs)}")
        exe = os.path.join(ROOT, "bin", "ffc-ffi-test")
        lines.append(f"build {exe}: cc_exe {os.path.join(ROOT, 'csrc', 'ffi', 'test_ffi.c')} | {lib}")
        defaults += [lib, exe]
        # legacy FFModel runtime API (csrc/ffi/flexflow_runtime_c.h): a separate
        # library, since its symbols overlap the graph API's (as in the reference)
        lines += ["rule cc_rt_exe",
                  f"  command = gcc -O2 -std=c11 -I{os.path.join(ROOT, 'csrc', 'ffi')} -o $out $in "
                  f"-L{os.path.join(PKG, 'lib')} -lflexflow_runtime_c -lm -Wl,-rpath,{os.path.join(PKG, 'lib')}",
                  "  description = CC $out"]
        ro = os.path.join("obj", "ffi", "flexflow_runtime_c.cc.o")
        lines.append(f"build {ro}: cxx {os.path.join(ROOT, 'csrc', 'ffi', 'flexflow_runtime_c.cc')}")
        # the GPU backing (csrc/ffdev) and the kernel objects it calls (not the
        # pybind bindings): the C API trains on the GPU when one is visible
        do = os.path.join("obj", "ffdev", "device_exec.cpp.o")
        lines.append(f"build {do}: hip {os.path.join(ROOT, 'csrc', 'ffdev', 'device_exec.cpp')}")
        lines.append(f"  hip_flags = $hip_flags {core_inc}")
        kobjs = []
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "kernels", "*.hip"))):
            o = os.path.join("obj", "kernels", os.path.basename(s) + ".o")
            if "kernels" not in targets:
                lines.append(f"build {o}: hip {s}")
            kobjs.append(o)
        lines += ["rule link_hip_so",
                  f"  command = $hipcc -shared --offload-arch={ARCH} -o $out $in -L{os.path.join(ROCM, 'lib')} "
                  "-lhipblaslt -lpthread",
                  "  description = LINK $out"]
        rlib = os.path.join(PKG, "lib", "libflexflow_runtime_c.so")
        lines.append(f"build {rlib}: link_hip_so {ro} {do} {' '.join(core_objs)} {' '.join(kobjs)}")
        rexe = os.path.join(ROOT, "bin", "ffc-runtime-c-test")
        lines.append(f"build {rexe}: cc_rt_exe {os.path.join(ROOT, 'csrc', 'ffi', 'test_runtime_c.c')} | {rlib}")
        defaults += [rlib, rexe]
    if "kernels" in targets:
        # csrc/runtime/arena.cpp -> lib/libffarena.so: the step's device arena,
        # loaded by torch.cuda.memory.CUDAPluggableAllocator (host code only)
        ao = os.path.join("obj", "runtime", "arena.cpp.o")
        lines.append(f"build {ao}: hip {os.path.join(ROOT, 'csrc', 'runtime', 'arena.cpp')}")
        alib = os.path.join(PKG, "lib", "libffarena.so")
        lines += ["rule link_arena",
                  f"  command = $hipcc -shared -o $out $in -L{os.path.join(ROCM, 'lib')} -lamdhip64",
                  "  description = LINK $out"]
        lines.append(f"build {alib}: link_arena {ao}")
        defaults.append(alib)
    if "replay" in targets:
        # csrc/runtime/replay.cpp -> _ffreplay: the native walker of segmented
        # distributed steps (hipGraph launches + c10d ProcessGroup collectives);
        # a host-only torch extension (libtorch / libtorch_hip, no device code)
        import torch
        from torch.utils import cpp_extension as cpp

        tinc = " ".join(f"-I{p}" for p in cpp.include_paths(device_type="cuda"))
        tlib = " ".join(f"-L{p}" for p in cpp.library_paths(device_type="cuda"))
        abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
        lines += [f"replay_flags = -O2 -std=c++17 -fPIC -DUSE_ROCM=1 -D__HIP_PLATFORM_AMD__=1 "
                  f"-DTORCH_EXTENSION_NAME=_ffreplay -DTORCH_API_INCLUDE_EXTENSION_H -D_GLIBCXX_USE_CXX11_ABI={abi} "
                  f"{tinc} {inc}",
                  "rule cxx_replay",
                  "  command = $cxx $replay_flags -MMD -MF $out.d -c $in -o $out",
                  "  depfile = $out.d",
                  "  deps = gcc",
                  "  description = CXX(torch) $in",
                  "rule link_replay",
                  f"  command = $cxx -shared -o $out $in {tlib} -lc10 -ltorch -ltorch_cpu -ltorch_python -lc10_hip "
                  "-ltorch_hip",
                  "  description = LINK $out"]
        ro = os.path.join("obj", "runtime", "replay.cpp.o")
        lines.append(f"build {ro}: cxx_replay {os.path.join(ROOT, 'csrc', 'runtime', 'replay.cpp')}")
        rso = os.path.join(PKG, "_ffreplay" + EXT)
        lines.append(f"build {rso}: link_replay {ro}")
        defaults.append(rso)
    if "asan" in targets:
        # host-code sanitizer build (ASan/UBSan for host code): the
        # C++ core + C ABI + native CLIs compiled with -fsanitize=address,undefined
        # into standalone executables under bin/asan/ (tests/test_sanitizers.py)
        san = "-O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined"
        lines += [f"san_flags = -std=c++17 -fPIC -Wall -Wno-unused-function {core_inc} "
                  f"-I{os.path.join(ROOT, 'csrc', 'ffi')} {san}",
                  "rule cxx_san",
                  "  command = $cxx $san_flags -MMD -MF $out.d -c $in -o $out",
                  "  depfile = $out.d",
                  "  deps = gcc",
                  "  description = CXX(asan) $in",
                  "rule cc_san",
                  f"  command = gcc -std=c11 {san} -I{os.path.join(ROOT, 'csrc', 'ffi')} -c $in -o $out",
                  "  description = CC(asan) $in",
                  "rule link_san",
                  f"  command = $cxx {san} -o $out $in -lpthread",
                  "  description = LINK(asan) $out"]
        san_objs = []
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "ffcore", "src", "*.cc"))):
            o = os.path.join("obj", "asan", os.path.basename(s) + ".o")
            lines.append(f"build {o}: cxx_san {s}")
            san_objs.append(o)
        fo = os.path.join("obj", "asan", "flexflow_c.cc.o")
        lines.append(f"build {fo}: cxx_san {os.path.join(ROOT, 'csrc', 'ffi', 'flexflow_c.cc')}")
        to = os.path.join("obj", "asan", "test_ffi.c.o")
        lines.append(f"build {to}: cc_san {os.path.join(ROOT, 'csrc', 'ffi', 'test_ffi.c')}")
        exe = os.path.join(ROOT, "bin", "asan", "ffc-ffi-test")
        lines.append(f"build {exe}: link_san {to} {fo} {' '.join(san_objs)}")
        defaults.append(exe)
        ro = os.path.join("obj", "asan", "flexflow_runtime_c.cc.o")
        lines.append(f"build {ro}: cxx_san {os.path.join(ROOT, 'csrc', 'ffi', 'flexflow_runtime_c.cc')}")
        rto = os.path.join("obj", "asan", "test_runtime_c.c.o")
        lines.append(f"build {rto}: cc_san {os.path.join(ROOT, 'csrc', 'ffi', 'test_runtime_c.c')}")
        # no HIP in the sanitizer build: the host-only make_device_backing
        hb = os.path.join("obj", "asan", "device_backing_host.cc.o")
        lines.append(f"build {hb}: cxx_san {os.path.join(ROOT, 'csrc', 'ffi', 'device_backing_host.cc')}")
        exe = os.path.join(ROOT, "bin", "asan", "ffc-runtime-c-test")
        lines.append(f"build {exe}: link_san {rto} {ro} {hb} {' '.join(san_objs)}")
        defaults.append(exe)
        for s in sorted(glob.glob(os.path.join(ROOT, "csrc", "tools", "*.cc"))):
            o = os.path.join("obj", "asan", "tool_" + os.path.basename(s) + ".o")
            lines.append(f"build {o}: cxx_san {s}")
            exe = os.path.join(ROOT, "bin", "asan", "ffc-" + os.path.basename(s)[:-3].replace("_", "-"))
            lines.append(f"build {exe}: link_san {o} {' '.join(san_objs)}")
            defaults.append(exe)
    lines.append("default " + " ".join(defaults))
    os.makedirs(BUILD, exist_ok=True)
    path = os.path.join(BUILD, "build.ninja")
    text = "\n".join(lines) + "\n"
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(targets: list[str] | None = None, jobs: int | None = None, verbose: bool = False) -> None:
    targets = targets or ["core", "kernels", "tools", "ffi", "replay"]
    write_ninja(targets)
    ninja = shutil.which("ninja")
    if ninja is None:
        try:
            import ninja as _ninja  # type: ignore

            ninja = os.path.join(_ninja.BIN_DIR, "ninja")
        except Exception as e:  # pragma: no cover
            raise RuntimeError("ninja not found") from e
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = [ninja, "-C", BUILD, f"-j{jobs}"]
    if verbose:
        cmd.append("-v")
    subprocess.run(cmd, check=True)


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("-")]
    build(args or None, verbose="-v" in sys.argv)
