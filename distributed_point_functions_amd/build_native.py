"""Builds the native pieces in-tree (no JIT cache, so they travel to the GPU box).

* ``distributed_point_functions_amd/lib/libdpf_hip.so`` -- HIP kernels + the C ABI
  of ``include/dpf_hip.h`` (hipcc, ``--offload-arch=gfx950``).
* ``distributed_point_functions_amd/lib/libdpf.so`` -- the host C++
  ``DistributedPointFunction`` (reference API) on top of that C ABI.
* ``distributed_point_functions_amd/lib/_dpf_host*.so`` -- pybind11 module over
  the host library (Python mirror used by tests and bench).
* ``oracle/liboracle_dpf.so`` -- the CPU parity oracle (test infrastructure).

Usage: ``python -m distributed_point_functions_amd.build_native [--only hip|host|oracle]``
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "distributed_point_functions_amd")
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
INCLUDE = os.path.join(ROOT, "include")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")

HIP_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-mcode-object-version=5", "-Wall", "-Wno-unused-function",
    # The AES rounds are LDS-latency bound: this scheduler keeps ~8-14 table
    # reads in flight per wave instead of 2-3 (tools/variant_bench.py, r04:
    # batched points 76 -> 89 G AES/s, expand 82 -> 84).
    "-mllvm", "-amdgpu-sched-strategy=iterative-ilp",
    # -DDPF_LEAF_QUADS (leaf quads, the last 8 AES of every 10 as ILP4) is
    # available but off: +1.9% same-box in tools/variant_bench.py, but it
    # spills 88 B/lane and the scratch traffic doubles the kernel's HBM bytes
    # (profiled r06: 16.5 GB/launch vs 8.9-10.7 GB).
]

# Translation units built with LLVM's default scheduler: with iterative-ilp,
# ROCm 7.2's greedy register allocator segfaults on the Mod32 key-sum kernel
# (batch_level_kernel<Mod32V, 2, true>, 128 VGPRs).
# dpf_expand_hybrid.hip: the bitsliced rounds need the default scheduler's
# register discipline (iterative-ilp: 228 VGPRs vs 175 at 2 waves per SIMD).
DEFAULT_SCHED_TUS = {"dpf_batch.hip", "dpf_expand_hybrid.hip", "dpf_expand_ws.hip"}


def _run(cmd, cwd=ROOT):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _files(d, exts):
    res = []
    for root, _, fs in os.walk(d):
        for f in fs:
            if f.endswith(exts):
                res.append(os.path.join(root, f))
    return res


def build_hip(force=False):
    """Each kernel translation unit is compiled to an object in parallel, then
    linked into one shared library."""
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, "libdpf_hip.so")
    kdir = os.path.join(CSRC, "kernels")
    srcs = sorted(f for f in _files(kdir, (".hip",)))
    hdrs = _files(kdir, (".h",)) + [os.path.join(INCLUDE, "dpf_hip.h")]
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    base_flags = [f for f in HIP_FLAGS if f != "-shared"]
    objs, procs = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            compile_flags = base_flags
            if os.path.basename(src) in DEFAULT_SCHED_TUS:
                compile_flags = [f for f in base_flags
                                 if f not in ("-mllvm", "-amdgpu-sched-strategy=iterative-ilp")]
            cmd = [HIPCC, *compile_flags, f"-I{INCLUDE}", "-c", src, "-o", obj]
            print("+", " ".join(cmd), flush=True)
            procs.append((cmd, subprocess.Popen(cmd, cwd=ROOT)))
    for cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    if force or procs or _stale(out, objs):
        _run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out])
    return out


def build_host(force=False):
    """Host C++ library (reference API) + pybind11 module."""
    host_dir = os.path.join(CSRC, "host")
    srcs = sorted(f for f in _files(host_dir, (".cc",)) if not f.endswith("_pybind.cc"))
    if not srcs:
        return None
    os.makedirs(LIBDIR, exist_ok=True)
    hdrs = _files(os.path.join(INCLUDE), (".h",)) + _files(host_dir, (".h",))
    out = os.path.join(LIBDIR, "libdpf.so")
    cxx = os.environ.get("CXX", "g++")
    common = ["-O2", "-std=c++20", "-fPIC", "-Wall", "-Wextra", "-Wno-unused-parameter",
              "-maes", "-msse4.1", f"-I{INCLUDE}"]
    if force or _stale(out, srcs + hdrs + [os.path.join(LIBDIR, "libdpf_hip.so")]):
        _run([cxx, *common, "-shared", *srcs, "-o", out, f"-L{LIBDIR}", "-ldpf_hip",
              "-Wl,-rpath,$ORIGIN"])
    pyb = os.path.join(host_dir, "dpf_pybind.cc")
    if os.path.exists(pyb):
        import pybind11
        suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
        mod = os.path.join(LIBDIR, "_dpf_host" + suffix)
        if force or _stale(mod, [pyb, out] + hdrs):
            _run([cxx, *common, "-shared", pyb, "-o", mod,
                  f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
                  f"-L{LIBDIR}", "-ldpf", "-ldpf_hip", "-Wl,-rpath,$ORIGIN"])
    return out


def build_oracle(force=False):
    odir = os.path.join(ROOT, "oracle")
    out = os.path.join(odir, "liboracle_dpf.so")
    if force or _stale(out, [os.path.join(odir, "dpf_oracle.c"), os.path.join(odir, "cpu_baseline.c")]):
        _run(["make", "-C", odir, "-B" if force else "liboracle_dpf.so"])
    return out


def build_tools(force=False):
    """C++ programs written against the drop-in API: the reference's benchmark
    suite restated (tools/dpf_benchmark.cc) and the C++ template tests
    (tests/cpp/dpf_api_test.cc)."""
    hdrs = _files(os.path.join(INCLUDE), (".h",))
    cxx = os.environ.get("CXX", "g++")
    for src, name in ((os.path.join(ROOT, "tools", "dpf_benchmark.cc"), "dpf_benchmark"),
                      (os.path.join(ROOT, "tests", "cpp", "dpf_api_test.cc"), "dpf_api_test")):
        out = os.path.join(LIBDIR, name)
        if force or _stale(out, [src, os.path.join(LIBDIR, "libdpf.so")] + hdrs):
            _run([cxx, "-O2", "-std=c++20", "-Wall", f"-I{INCLUDE}", src, "-o", out,
                  f"-L{LIBDIR}", "-ldpf", "-ldpf_hip", "-Wl,-rpath,$ORIGIN"])


def build_all(force=False):
    build_hip(force)
    build_host(force)
    build_tools(force)
    build_oracle(force)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["hip", "host", "oracle"])
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args(argv)
    if a.only == "hip":
        build_hip(a.force)
    elif a.only == "host":
        build_host(a.force)
    elif a.only == "oracle":
        build_oracle(a.force)
    else:
        build_all(a.force)


if __name__ == "__main__":
    sys.exit(main())
