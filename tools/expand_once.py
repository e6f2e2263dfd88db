#!/usr/bin/env python3
"""Config-2 expand kernel alone (one start seed, 29 levels, uint64, 2^30
outputs, random correction words) run --reps times: the program rocprofv3
profiles for the kernel A/B (tools/hyb_profile.sh).  Timing only."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from distributed_point_functions_amd import hip_abi as H
    H.load(require_gpu=True)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    keys = (0x5be037ccf6a03de5935f08d0a5b6a2fd, 0xef94b6aedebb026ce2ea1fe0f66f4d0b,
            0x05a5d1588c5423e346a31101b21d1c98)
    desc = H.value_desc([(H.LEAF_INT, 64, 0)], True, 2, 1)
    D = 29

    def rb(n):
        return torch.randint(-2**63, 2**63 - 1, (n, 2), dtype=torch.int64, device=dev, generator=g)
    seeds, cws, vcw = rb(1), rb(D), rb(2)
    ctrl = torch.zeros(1, dtype=torch.uint8, device=dev)
    cl = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    cr = torch.randint(0, 2, (D,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty((1 << 30) * 8, dtype=torch.uint8, device=dev)
    for _ in range(a.reps):
        H.expand(seeds, ctrl, cws, cl, cr, keys, desc, 2, vcw, 0, out=out)
    torch.cuda.synchronize()
    print("expand_once: done", flush=True)


if __name__ == "__main__":
    main()
