#!/usr/bin/env python3
"""Summarises one rocprofv3 collection directory (trace/ with --kernel-trace
--stats, and p*/ PMC passes, as written by tools/profile_workload.sh or
profiles/profile.sh) for one kernel into the profiles/<tag>_summary.json
format: per-launch counter averages, the sustained clock, LDS-pipe busy
fraction, VALU / LDS instructions per AES block and HBM write bytes (WRITE_SIZE
is in KiB on gfx950, MI355X_MICROARCH.md; GRBM_GUI_ACTIVE sums the 8 XCDs).

  python tools/pmc_summary.py <dir> <kernel substring> --aes N --bytes B [--tag t]
  python tools/pmc_summary.py <dir> <kernel substring> --bench-log <trace pass log> \
      --workload <bench.py workload tag> [--skip W | --total --passes P]

--bench-log takes the algorithmic AES / bytes / outputs per launch (or per
pass) from the bench.py JSON line the profiled command printed, and
--workload tags the summary so bench.py quotes it for that workload only.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

CUS = 256


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel", help="kernel name substring; alternatives separated by |")
    ap.add_argument("--aes", type=int, default=None, help="algorithmic AES blocks per launch")
    ap.add_argument("--bytes", type=int, default=None, help="algorithmic bytes written per launch")
    ap.add_argument("--bench-log", default=None,
                    help="log of the profiled bench.py run: its JSON line supplies --aes/--bytes/--leaves")
    ap.add_argument("--workload", default=None, help="bench.py workload tag this summary is for")
    ap.add_argument("--passes", type=int, default=1,
                    help="--total mode: the profiled run repeated the workload this many times "
                         "(warmup + timed steps); totals are divided by it")
    ap.add_argument("--tag", default="")
    ap.add_argument("--total", action="store_true",
                    help="sum every matching dispatch (a workload of many differently sized "
                         "launches, e.g. one heavy-hitters pass): --aes/--bytes are totals")
    ap.add_argument("--skip", type=int, default=0,
                    help="per-launch mode: drop the first N launches (bench.py's --warmup "
                         "steps) so avg_ns is the bench's timed region")
    ap.add_argument("--leaves", type=int, default=None,
                    help="outputs per launch (full domain; bench.py's profiled_traffic key)")
    a = ap.parse_args()
    a.kernel = a.kernel.replace("(anonymous namespace)::", "")
    res = {"tag": a.tag}
    if a.workload:
        res["workload"] = a.workload
    if a.bench_log:
        line = None
        for ln in open(a.bench_log, errors="replace"):
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
        if line is None:
            raise SystemExit(f"no bench.py JSON line in {a.bench_log}")
        roof = line.get("roofline", {})
        if a.aes is None:
            a.aes = int(roof.get("algorithmic_aes_per_launch") or roof.get("algorithmic_aes_per_pass"))
        if a.bytes is None:
            a.bytes = int(roof.get("algorithmic_bytes_per_launch") or 0)
        if a.leaves is None and line.get("config", {}).get("outputs_per_gpu"):
            a.leaves = int(line["config"]["outputs_per_gpu"])
        res["bench_launch_ms"] = roof.get("launch_ms") or roof.get("launch_ms_per_pass")
        res["bench_config"] = line.get("config", {}).get("workload")
    if a.aes is None or a.bytes is None:
        raise SystemExit("--aes and --bytes (or --bench-log) are required")
    # Per-launch mode keeps only the launches with the largest grid: a bench
    # run's spot checks call the same kernel on a few points.
    durs = []
    for f in glob.glob(os.path.join(a.dir, "trace", "*kernel_trace.csv")):
        for row in csv.DictReader(open(f)):
            if any(k in row["Kernel_Name"].replace("(anonymous namespace)::", "") for k in a.kernel.split("|")):
                durs.append((int(row["Grid_Size_X"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"]),
                             row["Kernel_Name"], int(row["Start_Timestamp"])))
    grid = max(d[0] for d in durs) if durs else None
    if durs:
        durs.sort(key=lambda d: d[3])
        sel = [d for g, d, _, _ in durs if a.total or g == grid]
        skipped = 0
        if not a.total and a.skip and len(sel) > a.skip:
            skipped, sel = a.skip, sel[a.skip:]
        res.update(kernel=durs[0][2], calls=len(sel), warmup_launches_skipped=skipped,
                   avg_ns=(sum(sel) / a.passes if a.total else sum(sel) / len(sel)),
                   min_ns=min(sel), max_ns=max(sel))
        if a.total:
            res["passes"] = a.passes
            # A pass of several kernels: `kernel` names them by share of the
            # pass's device time (largest first), `kernels` has the split.
            per_k = defaultdict(lambda: [0, 0])
            for _, d, name, _ in durs:
                per_k[name][0] += 1
                per_k[name][1] += d
            tot = sum(v[1] for v in per_k.values())
            order = sorted(per_k.items(), key=lambda kv: -kv[1][1])
            res["kernels"] = [{"kernel": k, "calls": v[0], "ns_per_pass": v[1] / a.passes,
                               "share": v[1] / tot} for k, v in order]
            res["kernel"] = " + ".join(k for k, _ in order)
    sums, launches = defaultdict(float), defaultdict(set)
    for f in glob.glob(os.path.join(a.dir, "p*", "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if (any(k in row["Kernel_Name"].replace("(anonymous namespace)::", "") for k in a.kernel.split("|"))
                    and (a.total or int(row["Grid_Size"]) == grid)):
                c = row["Counter_Name"]
                sums[c] += float(row["Counter_Value"])
                launches[c].add(row["Dispatch_Id"])
    per = {c: sums[c] / (a.passes if a.total else len(launches[c])) for c in sums}
    res["counters_per_launch"] = per
    aes = a.aes
    res["aes_blocks_per_launch"] = aes
    if a.leaves:
        res["leaves_per_launch"] = a.leaves
    if "avg_ns" in res:
        res["gaes_per_s"] = aes / res["avg_ns"]
    if "GRBM_GUI_ACTIVE" in per and "avg_ns" in res:
        cyc = per["GRBM_GUI_ACTIVE"] / 8
        res["effective_clock_ghz"] = cyc / res["avg_ns"]
        res["clk_per_aes_per_cu"] = cyc * CUS / aes
        if "SQ_INSTS_LDS" in per:
            res["lds_pipe_busy"] = per["SQ_INSTS_LDS"] * 2 / CUS / cyc
    if "SQ_INSTS_VALU" in per:
        res["valu_lane_ops_per_aes"] = per["SQ_INSTS_VALU"] * 64 / aes
    if "SQ_INSTS_LDS" in per:
        res["lds_lane_ops_per_aes"] = per["SQ_INSTS_LDS"] * 64 / aes
    if "WRITE_SIZE" in per:
        res["hbm_write_bytes"] = per["WRITE_SIZE"] * 1024
        if a.bytes > 0:
            res["algorithmic_write_bytes"] = a.bytes
            res["write_amplification"] = res["hbm_write_bytes"] / a.bytes
    if "FETCH_SIZE" in per:
        res["hbm_read_bytes_corrected"] = per["FETCH_SIZE"] * 1024 * 2
    if "hbm_write_bytes" in res:
        res["hbm_traffic_bytes"] = res["hbm_write_bytes"] + res.get("hbm_read_bytes_corrected", 0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
