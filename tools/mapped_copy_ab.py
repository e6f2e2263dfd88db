#!/usr/bin/env python3
"""A/B of the registration threshold for host ranges whose pages are already
mapped: dpf_hip_memcpy_h2d from, and dpf_hip_memcpy_d2h into, a
touched numpy buffer of 32-256 MiB, with DPF_HIP_REGISTER_MAPPED_MIB set per
process (32 = register from 32 MiB, 512 = the fresh-destination threshold,
i.e. bounce buffers below 512 MiB).  Prints one JSON line per (size, dir).

  python tools/mapped_copy_ab.py            # runs both settings as children
  python tools/mapped_copy_ab.py --child    # one setting (env), this process
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    import ctypes
    import numpy as np
    import torch
    from distributed_point_functions_amd import hip_abi as H
    lib = H.load(require_gpu=True)
    mib = os.environ.get("DPF_HIP_REGISTER_MAPPED_MIB")
    for size_mib in (32, 64, 128, 256):
        n = size_mib << 20
        host = np.ones(n, dtype=np.uint8)            # touched: pages mapped
        dev = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for name, fn in (("h2d", lambda: lib.dpf_hip_memcpy_h2d(
                              ctypes.c_void_p(dev.data_ptr()), host.ctypes.data_as(ctypes.c_void_p),
                              ctypes.c_size_t(n), None)),
                         ("d2h", lambda: lib.dpf_hip_memcpy_d2h(
                              host.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(dev.data_ptr()),
                              ctypes.c_size_t(n), None))):
            ts = []
            for _ in range(6):
                t0 = time.perf_counter()
                rc = fn()
                ts.append(time.perf_counter() - t0)
                assert rc == 0, rc
            ts = sorted(ts[1:])
            print(json.dumps({"mapped_register_min_mib": int(mib), "dir": name, "mib": size_mib,
                              "median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3,
                              "gb_per_s": n / ts[len(ts) // 2] / 1e9}), flush=True)


def main():
    if "--child" in sys.argv:
        return child()
    for mib in ("32", "512"):
        env = dict(os.environ, DPF_HIP_REGISTER_MAPPED_MIB=mib)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child"], env=env,
                           timeout=300)
        if r.returncode:
            raise SystemExit(r.returncode)


if __name__ == "__main__":
    main()
