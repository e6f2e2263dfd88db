#!/usr/bin/env python3
"""A/B of the octet expand kernel (default for whole-block integer leaves)
against expand_kernel (DPF_EXPAND_NO_OCTET=1) at config 2's shape (29 levels,
uint64, 2^30 outputs, random correction words, both parties): outputs must be
identical; prints both HIP-event times."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from distributed_point_functions_amd import hip_abi as H
    H.load(require_gpu=True)
    dev = torch.device("cuda")
    g = torch.Generator(device=dev)
    g.manual_seed(11)
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
    outs, times = [], []
    for variant in ("1", "0"):
        os.environ["DPF_EXPAND_NO_OCTET"] = variant
        for party in (0, 1):
            out = torch.empty((1 << 30) * 8, dtype=torch.uint8, device=dev)
            H.expand(seeds, ctrl, cws, cl, cr, keys, desc, 2, vcw, party, out=out)
            ev = [(H.Event(), H.Event()) for _ in range(3)]
            for a, b in ev:
                a.record()
                H.expand(seeds, ctrl, cws, cl, cr, keys, desc, 2, vcw, party, out=out)
                b.record()
            torch.cuda.synchronize()
            times.append((variant, party, float(np.mean([a.elapsed_ms(b) for a, b in ev]))))
            outs.append(out)
        if variant == "0":
            same = all(torch.equal(outs[i], outs[i + 2]) for i in (0, 1))
    print({"octet_identical_to_expand_kernel": same,
           "ms (no_octet, party)": times}, flush=True)


if __name__ == "__main__":
    main()
