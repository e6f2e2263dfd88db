#!/usr/bin/env python3
"""Summarises a profiles/profile.sh output directory into profiles/<tag>_summary.json
and profiles/<tag>_kernel_stats.csv (the rocprofv3 --stats table, committed).

Per-launch HBM traffic follows MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so fetched bytes = 2 * FETCH_SIZE * 1024 (upper estimate for
this kernel, whose reads are tiny); WRITE_SIZE * 1024 is exact for 16-B-per-lane
stores.  Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time.
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))


def per_kernel(path, match):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if match in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(tag, match="expand_kernel", aes_per_launch=None, leaves_per_launch=None):
    d = os.path.join(os.path.dirname(ROOT), "gpurun_out", f"prof_{tag}")
    stats = os.path.join(d, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(ROOT, f"{tag}_kernel_stats.csv"))
    kstats = [r for r in csv.DictReader(open(stats)) if match in r["Name"]][0]
    avg_ns = float(kstats["AverageNs"])
    c = {}
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, f"{sub}_counter_collection.csv")
        if sub.startswith("pmc") and os.path.exists(f):
            c.update(per_kernel(f, match))
    out = {"tag": tag, "kernel": kstats["Name"], "calls": int(kstats["Calls"]),
           "avg_ns": avg_ns, "counters_per_launch": c}
    if "GRBM_GUI_ACTIVE" in c:
        out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / avg_ns
    if "WRITE_SIZE" in c:
        out["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in c:
        out["hbm_read_bytes_corrected"] = 2 * c["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in c and "FETCH_SIZE" in c:
        out["hbm_traffic_bytes"] = out["hbm_write_bytes"] + out["hbm_read_bytes_corrected"]
    if aes_per_launch:
        out["aes_blocks_per_launch"] = aes_per_launch
        out["gaes_per_s"] = aes_per_launch / avg_ns
        if "SQ_INSTS_VALU" in c:
            out["valu_lane_ops_per_aes"] = c["SQ_INSTS_VALU"] * 64 / aes_per_launch
        if "SQ_INSTS_LDS" in c:
            out["lds_lane_ops_per_aes"] = c["SQ_INSTS_LDS"] * 64 / aes_per_launch
        if "effective_clock_ghz" in out:
            out["clk_per_aes_per_cu"] = 256 * out["effective_clock_ghz"] * avg_ns / aes_per_launch
    if leaves_per_launch:
        out["leaves_per_launch"] = leaves_per_launch
        out["algorithmic_write_bytes"] = leaves_per_launch * 8
        if "hbm_write_bytes" in out:
            out["write_amplification"] = out["hbm_write_bytes"] / out["algorithmic_write_bytes"]
    with open(os.path.join(ROOT, f"{tag}_summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--match", default="expand_kernel", help="substring of the kernel name")
    ap.add_argument("--aes", type=int, default=2 * (2**29 - 1) + 2**29,
                    help="algorithmic AES blocks per launch (default: config 2, D = 29)")
    ap.add_argument("--leaves", type=int, default=2**30,
                    help="output elements per launch (8 B each for the write figure)")
    a = ap.parse_args()
    main(a.tag, match=a.match, aes_per_launch=a.aes, leaves_per_launch=a.leaves)
