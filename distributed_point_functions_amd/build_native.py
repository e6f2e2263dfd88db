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
HIPCC = os.environ.get("DPF_HIPCC", os.path.join(ROCM, "bin", "hipcc"))

HIP_FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    "-mcode-object-version=5", "-Wall", "-Wno-unused-function",
    # The AES rounds are LDS-latency bound: this scheduler keeps ~8-14 table
    # reads in flight per wave instead of 2-3 (tools/variant_bench.py, r04:
    # batched points 76 -> 89 G AES/s, expand 82 -> 84).
    "-mllvm", "-amdgpu-sched-strategy=iterative-ilp",
]

# Translation units built with LLVM's default scheduler: with iterative-ilp,
# ROCm 7.2's greedy register allocator segfaults on the Mod32 key-sum kernel
# (batch_level_kernel<Mod32V, 2, true>, 128 VGPRs).
DEFAULT_SCHED_TUS = {"dpf_batch.hip"}


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


# The compiler workaround the kernels depend on (DESIGN.md "Build"): ROCm
# 7.2's iterative-ilp scheduler segfaults on the octet expand kernel unless
# aes_core.h's encryptN puts a sched_barrier after every DPF_LAST_ROUND_FENCE
# last-round chains, and its register allocator crashes on dpf_batch.hip
# (DEFAULT_SCHED_TUS).  A hipcc crash on a TU built with iterative-ilp is
# reported as that known issue and the TU is rebuilt with the default
# scheduler (6-8% slower kernels, so the fallback is announced, not silent).
ILP_FLAGS = ("-mllvm", "-amdgpu-sched-strategy=iterative-ilp")
CRASH_MARKERS = ("PLEASE submit a bug report", "Stack dump", "Segmentation fault",
                 "crash backtrace", "LLVM ERROR")


def fence_setting(src: str) -> int:
    """DPF_LAST_ROUND_FENCE in effect for a kernel TU: its own #define, else
    aes_core.h's default."""
    import re
    for path in (src, os.path.join(CSRC, "kernels", "aes_core.h")):
        m = re.search(r"^#define DPF_LAST_ROUND_FENCE (\d+)", open(path).read(), re.M)
        if m:
            return int(m.group(1))
    return 0


def _crashed(rc: int, err: str) -> bool:
    return rc < 0 or rc >= 128 or any(m in err for m in CRASH_MARKERS)


def _compile_tu(cmd, src, uses_ilp):
    """Runs one hipcc compile; on an iterative-ilp compiler crash, reports the
    known issue and retries without that scheduler.  Returns the scheduler used."""
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True)
    sys.stdout.write(p.stdout)
    sys.stderr.write(p.stderr)
    if p.returncode == 0:
        return "iterative-ilp" if uses_ilp else "default"
    if uses_ilp and _crashed(p.returncode, p.stderr):
        print(f"build_native: KNOWN ISSUE: hipcc crashed compiling {os.path.basename(src)} "
              f"with -amdgpu-sched-strategy=iterative-ilp (ROCm 7.2 scheduler/regalloc crash; "
              f"DPF_LAST_ROUND_FENCE={fence_setting(src)}, DESIGN.md 'Build').  Rebuilding it "
              f"with the default scheduler (measured 6-8% slower kernels).", flush=True)
        cmd2 = [c for c in cmd if c not in ILP_FLAGS]
        p2 = subprocess.run(cmd2, cwd=ROOT, capture_output=True, text=True)
        sys.stdout.write(p2.stdout)
        sys.stderr.write(p2.stderr)
        if p2.returncode == 0:
            return "default (fallback after iterative-ilp crash)"
        raise subprocess.CalledProcessError(p2.returncode, cmd2)
    raise subprocess.CalledProcessError(p.returncode, cmd)


def build_hip(force=False):
    """Each kernel translation unit is compiled to an object in parallel, then
    linked into one shared library.  build/hip/build_manifest.json records the
    scheduler and last-round fence of every TU."""
    from concurrent.futures import ThreadPoolExecutor
    import json
    os.makedirs(LIBDIR, exist_ok=True)
    out = os.path.join(LIBDIR, "libdpf_hip.so")
    kdir = os.path.join(CSRC, "kernels")
    srcs = sorted(f for f in _files(kdir, (".hip",)))
    hdrs = _files(kdir, (".h",)) + [os.path.join(INCLUDE, "dpf_hip.h")]
    objdir = os.path.join(ROOT, "build", "hip")
    os.makedirs(objdir, exist_ok=True)
    base_flags = [f for f in HIP_FLAGS if f != "-shared"]
    manifest_path = os.path.join(objdir, "build_manifest.json")
    try:
        manifest = json.load(open(manifest_path))
    except (OSError, ValueError):
        manifest = {}
    objs, jobs = [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + hdrs):
            compile_flags = base_flags
            uses_ilp = os.path.basename(src) not in DEFAULT_SCHED_TUS
            if not uses_ilp:
                compile_flags = [f for f in base_flags if f not in ILP_FLAGS]
            cmd = [HIPCC, *compile_flags, f"-I{INCLUDE}", "-c", src, "-o", obj]
            print("+", " ".join(cmd), flush=True)
            jobs.append((src, cmd, uses_ilp))
    with ThreadPoolExecutor(max_workers=max(1, len(jobs))) as pool:
        futs = [(src, pool.submit(_compile_tu, cmd, src, ilp)) for src, cmd, ilp in jobs]
        for src, f in futs:
            manifest[os.path.basename(src)] = {"scheduler": f.result(),
                                               "last_round_fence": fence_setting(src)}
    if jobs:
        json.dump(manifest, open(manifest_path, "w"), indent=1, sort_keys=True)
        for tu, m in sorted(manifest.items()):
            print(f"build_native: {tu}: scheduler={m['scheduler']}, "
                  f"DPF_LAST_ROUND_FENCE={m['last_round_fence']}", flush=True)
    if force or jobs or _stale(out, objs):
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
