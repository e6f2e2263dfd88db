"""A/B of dynamic 64-item chunks (take_chunk) against the fixed grid-stride
share in hash_kernel (dpf_hip_hash) and eval_paths_kernel (dpf_hip_eval_paths).

Both variants run in one process, alternating, timed with HIP events on the
current stream; DPF_HASH_DYNAMIC / DPF_PATHS_DYNAMIC are read per launch.
Usage (GPU box, repo root): python tools/hash_paths_ab.py [--rounds 3]
Prints one line per run: <kernel> <variant> ms G AES/s.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_point_functions_amd import hip_abi as H
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--hash-log", type=int, default=26)
    ap.add_argument("--paths-log", type=int, default=24)
    ap.add_argument("--levels", type=int, default=64)
    a = ap.parse_args()
    H.load(require_gpu=True)
    g = torch.Generator(device="cuda").manual_seed(1)
    n = 1 << a.hash_log
    blocks = torch.randint(-2**62, 2**62, (n, 2), dtype=torch.int64, device="cuda", generator=g)
    out = torch.empty_like(blocks)
    m = 1 << a.paths_log
    seeds = torch.randint(-2**62, 2**62, (m, 2), dtype=torch.int64, device="cuda", generator=g)
    paths = torch.randint(-2**62, 2**62, (m, 2), dtype=torch.int64, device="cuda", generator=g)
    ctrl = torch.randint(0, 2, (m,), dtype=torch.uint8, device="cuda", generator=g)
    cws = torch.randint(-2**62, 2**62, (a.levels, 2), dtype=torch.int64, device="cuda", generator=g)
    cl = torch.randint(0, 2, (a.levels,), dtype=torch.uint8, device="cuda", generator=g)
    cr = torch.randint(0, 2, (a.levels,), dtype=torch.uint8, device="cuda", generator=g)
    s_out, c_out = torch.empty_like(seeds), torch.empty_like(ctrl)

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    runs = [("hash", "DPF_HASH_DYNAMIC", n,
             lambda: H.hash_blocks(blocks, 0, out=out)),
            ("paths", "DPF_PATHS_DYNAMIC", m * a.levels,
             lambda: H.eval_paths(seeds, ctrl, paths, cws, cl, cr, 0, 1, s_out, c_out))]
    for _ in range(a.rounds):
        for name, env, aes, fn in runs:
            for dyn in ("1", "0"):
                os.environ[env] = dyn
                ms = timed(fn)
                print(f"{name} {'dynamic' if dyn == '1' else 'fixed'} {ms:.3f} ms "
                      f"{aes / ms / 1e6:.1f} G AES/s", flush=True)


if __name__ == "__main__":
    main()
