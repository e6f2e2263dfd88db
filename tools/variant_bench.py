#!/usr/bin/env python3
"""Times the hot kernels of one build of libdpf_hip.so (DPF_HIP_LIB=<path>) on
synthetic inputs: the fused expand kernel at config 2 (one start seed, 29
levels, uint64, 2^30 outputs), the batched point kernel at 1/16 of config 4
(2^16 keys x 2^10 points, 127 levels) and the bare MMO hash (2^28 blocks).
Inputs are random correction words: timing only, parity is the tests' job.
Prints one JSON line: G AES-128 blocks/s per kernel (HIP events).

  python tools/variant_bench.py [--lib path ...]   (one subprocess per lib)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_one():
    import ctypes
    import numpy as np
    import torch
    from distributed_point_functions_amd import hip_abi as H
    L = H.load(require_gpu=True)
    L.dpf_hip_eval_points_batch.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
        [ctypes.c_void_p] * 12
    dev = torch.device("cuda")
    s = torch.cuda.current_stream()
    g = torch.Generator(device=dev)
    g.manual_seed(7)

    def rand_blocks(n):
        return torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device=dev, generator=g)

    def timed(fn, reps=3):
        fn()
        ev = [(H.Event(), H.Event()) for _ in range(reps)]
        for a, b in ev:
            a.record(s)
            fn()
            b.record(s)
        torch.cuda.synchronize()
        return float(np.mean([a.elapsed_ms(b) for a, b in ev]))

    res = {}
    keys = (0x5be037ccf6a03de5935f08d0a5b6a2fd, 0xef94b6aedebb026ce2ea1fe0f66f4d0b,
            0x05a5d1588c5423e346a31101b21d1c98)
    desc = H.value_desc([(H.LEAF_INT, 64, 0)], True, 2, 1)
    # expand, config 2
    D = 29
    seeds = rand_blocks(1)
    ctrl = torch.zeros(1, dtype=torch.uint8, device=dev)
    cws = rand_blocks(D)
    cl = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    cr = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    vcw = rand_blocks(2)
    out = torch.empty((1 << 30) * 8, dtype=torch.uint8, device=dev)
    ms = timed(lambda: H.expand(seeds, ctrl, cws, cl, cr, keys, desc, 2, vcw, 0, out=out))
    res["expand_ms"] = ms
    res["expand_gaes"] = (2 * (2**D - 1) + 2**D) / ms / 1e6
    del out
    # expand from 5 start seeds x 27 levels (5 * 2^28 uint64 outputs): with
    # S = 9 the 5 * 2^18 items divide evenly over 1024- and 640-thread
    # workgroups alike (variants built with -DDPF_FORCE_S=9)
    D5 = 27
    seeds5 = rand_blocks(5)
    ctrl5 = torch.tensor([0, 1, 0, 1, 1], dtype=torch.uint8, device=dev)
    out = torch.empty(5 * (1 << 28) * 8, dtype=torch.uint8, device=dev)
    ms = timed(lambda: H.expand(seeds5, ctrl5, cws[:D5], cl[:D5], cr[:D5], keys, desc, 2, vcw, 0,
                                out=out))
    res["expand5_ms"] = ms
    res["expand5_gaes"] = 5 * (2 * (2**D5 - 1) + 2**D5) / ms / 1e6
    del out
    # batched points, 2^16 keys x 2^10 points, log 128
    nk, ppk, Lv = 1 << 16, 1 << 10, 127
    kseed = rand_blocks(nk)
    party = torch.zeros(nk, dtype=torch.uint8, device=dev)
    kcw = rand_blocks(nk * Lv)
    kcl = torch.randint(0, 2, (nk * Lv,), dtype=torch.uint8, device=dev, generator=g)
    kcr = torch.randint(0, 2, (nk * Lv,), dtype=torch.uint8, device=dev, generator=g)
    kvcw = rand_blocks(nk * 2)
    pts = rand_blocks(nk * ppk)
    pout = torch.empty(nk * ppk * 8, dtype=torch.uint8, device=dev)
    kl, kr, kv = (H.aes_key(k) for k in keys)

    def pts_call():
        H.check(L.dpf_hip_eval_points_batch(nk, ppk, 0, Lv, Lv, 1, kseed.data_ptr(), party.data_ptr(),
                                            pts.data_ptr(), kcw.data_ptr(), kcl.data_ptr(),
                                            kcr.data_ptr(), ctypes.byref(kl), ctypes.byref(kr),
                                            ctypes.byref(kv), ctypes.byref(desc), kvcw.data_ptr(),
                                            pout.data_ptr(), H._stream()))
    ms = timed(pts_call)
    res["points_ms"] = ms
    res["points_gaes"] = nk * ppk * (Lv + 1) / ms / 1e6
    del pts, pout
    # bare hash
    n = 1 << 28
    blocks = rand_blocks(n)
    hout = torch.empty_like(blocks)
    ms = timed(lambda: H.hash_blocks(blocks, keys[2], out=hout))
    res["hash_gaes"] = n / ms / 1e6
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", nargs="*", default=None)
    ap.add_argument("--one", action="store_true")
    a = ap.parse_args()
    if a.one:
        return run_one()
    libs = a.lib or [os.path.join(ROOT, "distributed_point_functions_amd", "lib", "libdpf_hip.so")]
    for lib in libs:
        env = dict(os.environ, DPF_HIP_LIB=os.path.abspath(lib))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--one"], env=env,
                           capture_output=True, text=True, timeout=600)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(os.path.basename(lib), line[0] if line else ("FAILED rc=%d %s" % (r.returncode, r.stderr[-500:])),
              flush=True)


if __name__ == "__main__":
    main()
