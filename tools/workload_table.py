#!/usr/bin/env python3
"""Prints DESIGN.md section 5's all-workload table from a round's bench lines
(profiles/<tag>/bench_<tag>_<workload>.json and, for config 2,
profiles/<tag>_bench.json -- copied from tools/round_evidence.sh's gpurun_out/;
rounds up to r15: profiles/<tag>_<workload>_bench.json), so the table quotes
exactly the committed evidence.  The last column is the sustained clock the
line measured inside its own launches (in-kernel stamps, r16) or, for older
lines, the clock of the same lease's profile.

  python tools/workload_table.py r16
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ROWS = [
    # (bench file suffix, label, result formatter)
    ("full_domain", "config 2 full domain (2^30 uint64)",
     lambda d: f"{d['value'] / 1e9:.1f} G leaves/s, {d['ms_per_step']:.2f} ms per step"),
    ("config1", "config 1 full domain (2^20 uint64, latency mode)",
     lambda d: f"{d['value'] / 1e9:.1f} G leaves/s, {d['ms_per_step'] * 1e3:.1f} us per step"),
    ("full_domain_u128", "config 3 shard (2^31 uint128 per GPU)",
     lambda d: f"{d['value'] / 1e9:.1f} G leaves/s, {d['ms_per_step']:.1f} ms"),
    ("tuple_u32", "Tuple<uint32_t, uint32_t> full domain (2^30)",
     lambda d: f"{d['value'] / 1e9:.1f} G leaves/s, {d['ms_per_step']:.2f} ms"),
    ("tuple_mod", "Tuple<IntModN32 x 2> full domain (2^30)",
     lambda d: f"{d['value'] / 1e9:.1f} G leaves/s, {d['ms_per_step']:.1f} ms (2 value blocks per leaf)"),
    ("evaluate_at", "config 4 EvaluateAt (2^20 keys x 2^10, log 128)",
     lambda d: f"{d['value'] / 1e6:.0f} M points/s, {d['ms_per_step'] / 1e3:.2f} s"),
    ("evaluate_at_sum", "config 4, summed over keys",
     lambda d: f"{d['value'] / 1e6:.0f} M points/s"),
    ("heavy_hitters", "config 5b heavy hitters (one pass, both servers, expansion cache)",
     lambda d: f"{d['ms_per_step'] / 1e3:.1f} s, {d['value'] / 1e9:.1f} G prefix evals/s"),
    ("dcf", "DCF (2^16 keys x 2^10, log 64)",
     lambda d: f"{d['value'] / 1e6:.0f} M evals/s, {d['ms_per_step']:.1f} ms"),
]


def cpu(d):
    c = d.get("cpu_baseline") or {}
    if not c:
        return "—"
    v, u = c["value"], c["unit"]
    if v >= 1e8:
        return f"{v / 1e9:.2f} G {u}"
    if v >= 1e5:
        return f"{v / 1e6:.1f} M {u}"
    return f"{v:.0f} {u}"


def bench_path(tag: str, suffix: str) -> str:
    for p in ((f"{tag}_bench.json",) if suffix == "full_domain" else ()) + (
            os.path.join(tag, f"bench_{tag}_{suffix}.json"), f"{tag}_{suffix}_bench.json"):
        if os.path.exists(os.path.join(ROOT, "profiles", p)):
            return os.path.join(ROOT, "profiles", p)
    raise FileNotFoundError(f"no {tag} bench line for {suffix} under profiles/")


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r15"
    print("| workload | result | G AES/s | VALU roofline | clock (GHz) | CPU baseline (16 host threads) |")
    print("|---|---|---|---|---|---|")
    for suffix, label, fmt in ROWS:
        d = json.loads(open(bench_path(tag, suffix)).read().strip().splitlines()[-1])
        r = d.get("roofline", {})
        ghz = r.get("sustained_clock_ghz") or (r.get("pmc") or {}).get("sustained_clock_ghz")
        print(f"| {label} | {fmt(d)} | {r.get('achieved', 0):.1f} | {r.get('frac', 0):.3f} | "
              f"{ghz:.2f} | {cpu(d)} |" if ghz else
              f"| {label} | {fmt(d)} | {r.get('achieved', 0):.1f} | {r.get('frac', 0):.3f} | — | {cpu(d)} |")


if __name__ == "__main__":
    main()
