#!/usr/bin/env python3
"""Headline benchmark: full-domain DPF evaluation of a 2^30-output uint64 domain.

Metric (BASELINE.json): "DPF leaf evals/sec, full-domain 2^30 uint64 at
1/2/4/8 GPUs; AES blocks/s" -- configs[1]: DpfParameters{log_domain_size=30,
value_type=uint64}, one key, EvaluateUntil(0, {}, ctx).

One *step* goes through the product API exactly as a caller would:
`DistributedPointFunction.evaluate_shard_to_device(0, rank, N, ctx, out)` on a
fresh EvaluationContext (the drop-in for EvaluateUntil(0, {}, ctx) with the
outputs left in HBM).  Inside it the host
library validates the context, uploads the correction words (a few KiB), and
launches the fused gfx950 expand kernel (ExpandSeeds + HashExpandedSeeds +
value correction) that writes 2^30 * 8 B = 8 GiB of corrected outputs to HBM.
Keys are generated on the CPU (out of scope for the GPU) before
the timed region.  The PCIe-inclusive host-output rate (`--host-output`,
below) is reported beside it, never as `value`.

Multi-GPU (distributed_point_functions_amd/sharding.py): the
metric's configuration is ONE 2^30-output domain at 1/2/4/8 GPUs, so the
default is strong scaling by subtree prefix: with N = 2^k ranks, rank r
path-walks the top k tree levels along the bits of r and expands its own
2^(30-k)-output subtree; `value` = 2^30 outputs / the max-over-ranks step
time.  `--scaling weak` keeps 2^30 outputs per GPU (domain 2^(30+k)); the
uint128 workload (config 3: 2^34 outputs over 8 GPUs = 2^31 per GPU) is weak
by default.  No collective on the data path; one all_reduce(MAX) of the step
time outside the timed region.  `--rehearse-world W` runs, in one process on
one GPU, exactly the shard rank 0 of a W-rank run evaluates (the per-rank
kernel and fixed per-step host cost at that shard size).

The line also carries, beside `value` and never in it:
* `roofline.sustained_clock_ghz` / `clk_per_aes_per_cu`: the shader clock the
  timed launches themselves ran at (s_memtime / s_memrealtime stamps of every
  workgroup, dpf_hip_clock_probe), so a box can be told from a regression;
* `api_level` (configs 2 and 3, N = 1; `--no-host-output` skips it): the
  reference's own call shape, EvaluateUntil<uint64_t / absl::uint128>(0, {},
  ctx) returning a std::vector in host memory (the device kernel + the D2H
  copy into the caller's vector), timed on the same key -- PCIe-inclusive.

Run: python bench.py [--gpus N --steps K --warmup W]
     python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

LOG_PER_GPU = 30          # 2^30 uint64 outputs per GPU (BASELINE.json configs[1])
# AES-128 rooflines (DESIGN.md "Roofline"), 256 CUs at 2.4 GHz:
#  * VALU (the north_star's "integer-VALU AES roofline", the `roofline` object):
#    C_AES = 320 lane-ops/block (10 rounds x (16 byte extractions + 16 XOR
#    combines)) at 4 SIMD-32 x 32 lanes = 128 lane-ops/clk/CU -> 2.5 clk/block/CU
#    -> 245.8 G blocks/s.
#  * LDS (`roofline_lds`, the bound of the T-table design): 160 conflict-free
#    ds_read_b32 lookups = 640 B at 128 B/clk/CU -> 5 clk/block/CU -> 122.9 G.
#  * measured LDS ceiling (`roofline_lds_measured`): conflict-free random
#    ds_read_b32 lookups in this layout sustain 31.0 lanes/clk/CU of the 32
#    when every wave takes its work in chunks (tools/lds_ceiling_microbench.hip,
#    profiles/r16/lds_ceiling.txt; r11's 26.3 with fixed per-wave shares
#    included the launch's staggered tail) -> 31.0 x 256 x 2.4 GHz / 160 =
#    119.0 G blocks/s at the nominal clock.
AES_VALU_PEAK_GBLOCKS = 245.8
AES_LDS_PEAK_GBLOCKS = 122.9
AES_LDS_MEASURED_GBLOCKS = 119.0
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md
METRIC = "DPF leaf evals/sec, full-domain 2^30 uint64 at 1/2/4/8 GPUs; AES blocks/s"
KERNEL = "expand_octet_kernel<FastIntLeaf<64, false> >"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 20; 1 for heavy_hitters, whose step is a full pass)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 3; 1)")
    ap.add_argument("--log-domain", type=int, default=LOG_PER_GPU,
                    help="log2 outputs: of the whole domain (strong scaling) or per GPU (weak); "
                         "default 30 = the BASELINE config (31 per GPU for full_domain_u128)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-output", dest="host_output", action="store_true", default=True,
                    help="full_domain / full_domain_u128 at N = 1 (default on): also time the "
                         "drop-in API call that returns host memory, EvaluateUntil<T>(0, {}, ctx) "
                         "-> std::vector<T> (reported in `api_level`, never as `value`)")
    ap.add_argument("--no-host-output", dest="host_output", action="store_false")
    ap.add_argument("--scaling", choices=["strong", "weak"], default=None,
                    help="full_domain*: strong = one 2^log-domain split over the N GPUs (default; "
                         "the metric's configuration), weak = 2^log outputs per GPU (default for "
                         "full_domain_u128, whose config 3 is 2^31 outputs per GPU x 8)")
    ap.add_argument("--rehearse-world", type=int, default=None,
                    help="full_domain*: one process evaluates the shard rank 0 of a W-rank run "
                         "would (per-rank kernel time and fixed per-step cost at that size)")
    ap.add_argument("--host-output-reps", type=int, default=3)
    ap.add_argument("--cpu-chunks", type=int, default=32,
                    help="CPU baseline sample = this many 2^24-output subtrees of the same key")
    ap.add_argument("--workload", default="full_domain",
                    choices=["full_domain", "full_domain_u128", "full_domain_tuple", "evaluate_at",
                             "evaluate_at_sum",
                             "synthetic_hierarchical", "synthetic_hierarchical_device",
                             "synthetic_direct", "heavy_hitters", "dcf"],
                    help="full_domain = BASELINE configs[1] (the headline); full_domain_u128 = "
                         "configs[2] (2^31 uint128 outputs per GPU, 2^34 over 8 GPUs); "
                         "evaluate_at(_sum) = configs[3] (2^20 keys x 2^10 points, log 128)")
    ap.add_argument("--tuple-type", default="intmodn32x2", choices=["intmodn32x2", "u32x2"],
                    help="full_domain_tuple: Tuple<IntModN<uint32_t, 2^32-5> x 2> (Moller-Granlund "
                         "sampling from two blocks) or Tuple<uint32_t, uint32_t> (direct)")
    ap.add_argument("--keys-log", type=int, default=20, help="evaluate_at: log2 keys (all ranks)")
    ap.add_argument("--domain", type=int, default=32, help="synthetic_*: log2 domain (32 or 128)")
    ap.add_argument("--distribution", default="uniform", choices=["0.1", "0.5", "uniform"],
                    help="synthetic_*: 90%% of nonzeros in the first 10%%/50%% of the domain, or uniform")
    ap.add_argument("--points-log", type=int, default=10, help="evaluate_at: log2 points per key")
    ap.add_argument("--dcf-keys-log", type=int, default=16, help="dcf: log2 keys")
    ap.add_argument("--dcf-log-domain", type=int, default=64, help="dcf: log2 comparison domain")
    ap.add_argument("--top-k", type=int, default=1024,
                    help="heavy_hitters: candidates kept per level (children = 4 x top-k)")
    args = ap.parse_args()
    long_step = args.workload == "heavy_hitters"
    if args.steps is None:
        args.steps = 1 if long_step else 20
    if args.warmup is None:
        args.warmup = 1 if long_step else 3
    if args.scaling is None:
        args.scaling = "weak" if args.workload == "full_domain_u128" else "strong"
    if args.rehearse_world is not None and (args.gpus != 1 or not args.workload.startswith("full_domain")):
        raise SystemExit("--rehearse-world runs one full_domain* process (--gpus 1)")
    return args


def tree_aes_per_launch(depth: int, blocks_needed: int = 1) -> int:
    """AES-128 blocks one full-subtree expansion computes: two PRG calls per
    inner node (left/right children) plus `blocks_needed` value hashes per leaf
    seed."""
    return 2 * ((1 << depth) - 1) + blocks_needed * (1 << depth)


def _int_of(v) -> int:
    """Value.Integer -> int (uint64 or uint128 form)."""
    if v.integer.WhichOneof("value") == "value_uint128":
        return v.integer.value_uint128.high << 64 | v.integer.value_uint128.low
    return int(v.integer.value_uint64)


def baseline_threads() -> int:
    """Host threads for the CPU baselines: the cores this process may run on
    (sched_getaffinity), capped by OMP_NUM_THREADS -- the GPU box exports the
    per-GPU CPU share there (16) and its rules cap worker pools at that share."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(cap))) if cap and cap.isdigit() else n


CPU_THREADS = baseline_threads()   # 16 on the GPU box (its per-GPU CPU share)


def host_cpu(threads: int = None) -> dict:
    """CPU model and logical CPU count of the host the baseline ran on."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"model": model, "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "threads_used": threads if threads is not None else CPU_THREADS}


def cgroup_cpus():
    """CPUs the host's cgroup lets this process use (cpu.max quota / period),
    or None without a quota: the GPU box's share is 16 of its 256 CPUs."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def all_cores_sample(work, items, unit: str, budget_s: float = 8.0) -> dict:
    """The same CPU work on every host CPU the process may run on
    (sched_getaffinity), as SURVEY.md 8d asks beside the per-GPU share; the
    cgroup quota that bounds it is reported with it."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    units, dt, done = run_cpu_pool(work, items, threads=n, budget_s=budget_s)
    return {"value": units / dt, "unit": unit, "threads": n, "cgroup_cpu_quota": cgroup_cpus(),
            "sample": f"{done} work items, {dt:.1f} s wall on {n} host threads"}


def run_cpu_pool(work, items, threads: int = CPU_THREADS, budget_s: float = 15.0):
    """Runs work(item) -> units over `items` on `threads` host threads (the
    oracle's C calls release the GIL), submitting new items only while the
    wall time is under `budget_s`.  Returns (units done, wall seconds, items)."""
    from concurrent.futures import FIRST_COMPLETED, ThreadPoolExecutor, wait
    it = iter(items)
    units, n_items = 0, 0
    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads) as pool:
        pending = set()
        for _ in range(threads):
            nxt = next(it, None)
            if nxt is None:
                break
            pending.add(pool.submit(work, nxt))
        while pending:
            done, pending = wait(pending, return_when=FIRST_COMPLETED)
            for f in done:
                units += f.result()
                n_items += 1
                if time.perf_counter() - t0 < budget_s:
                    nxt = next(it, None)
                    if nxt is not None:
                        pending.add(pool.submit(work, nxt))
    return units, time.perf_counter() - t0, n_items


def _leaf_ints(v) -> list:
    """A proto Value flattened to its leaf integers (the oracle's value form)."""
    which = v.WhichOneof("value")
    if which == "tuple":
        return [x for e in v.tuple.elements for x in _leaf_ints(e)]
    iv = getattr(v, which)
    if iv.WhichOneof("value") == "value_uint128":
        return [iv.value_uint128.high << 64 | iv.value_uint128.low]
    return [int(iv.value_uint64)]


def cpu_baseline(key, log_domain: int, chunks: int, bits: int = 64, vt=None):
    """The oracle (C restatement of dpf/distributed_point_function.cc:271-349,
    OpenSSL AES-NI in 64-block batches) on the SAME workload, on CPU_THREADS host
    threads: the 2^24-output subtrees of the benchmark key, each walked to its
    root (EvaluateSeeds) then expanded + hashed + corrected, until a 20 s wall
    budget is spent (the whole domain fits in it on the GPU box).  `chunks` is
    kept for the command line and unused."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    vt = vt or ("int", bits)
    P = O.OracleParams([(log_domain, vt, 0)])
    epb = O.elements_per_block(vt)
    sub = 18 - (epb.bit_length() - 1)         # 2^18 outputs per work item
    b = P.blocks_needed[0]
    T = P.hierarchy_to_tree[0]
    top = T - sub
    # The product DpfKey (proto) restated as the oracle's key dict.
    k = {"seed": key.seed.high << 64 | key.seed.low, "party": key.party,
         "cws": [(c.seed.high << 64 | c.seed.low, int(c.control_left), int(c.control_right),
                  None) for c in key.correction_words],
         "last_vc": [_leaf_ints(v) for v in key.last_level_value_correction]}
    vcw = O._value_correction(P, k, 0)
    cs_top, cl_top, cr_top = O._cw_arrays(k, 0, top)
    cs, cl, cr = O._cw_arrays(k, top, T)
    # Every 2^18-output subtree of the domain is one work item (the whole
    # workload when the time budget allows), spread over the host threads.
    n_sub = 1 << top

    def work(c):
        seed, ctrl = O.evaluate_seeds(O.blocks_from_ints([k["seed"]]),
                                      np.array([k["party"]], np.uint8),
                                      O.blocks_from_ints([c]), cs_top, cl_top, cr_top)
        es, ec = O.expand_seeds(seed, ctrl, cs, cl, cr)
        return O.hash_correct(vt, es, ec, b, P.cepb(0), vcw, k["party"]).shape[0]

    leaves, dt, done = run_cpu_pool(work, range(n_sub), budget_s=20.0)
    # SURVEY.md 8d also asks for the single-threaded rate (the reference is
    # single-threaded): a 4 s sample on one thread.
    leaves1, dt1, done1 = run_cpu_pool(work, range(n_sub), threads=1, budget_s=4.0)
    return {"value": leaves / dt, "unit": "leaves/s", "cores": CPU_THREADS, "kind": "port",
            "single_thread_value": leaves1 / dt1,
            "all_cores": all_cores_sample(work, range(n_sub), "leaves/s"),
            "single_thread_sample": f"{done1} subtrees of 2^18 outputs, {dt1:.1f} s on 1 thread",
            "host": host_cpu(),
            "sample": f"{done} of the {n_sub} subtrees of 2^18 {vt} outputs of the benchmark "
                      f"key (2^{log_domain} domain): EvaluateSeeds to each subtree root, then "
                      f"ExpandSeeds+HashExpandedSeeds+correction (oracle over OpenSSL AES-NI); "
                      f"{dt:.1f} s wall on {CPU_THREADS} host threads",
            "aes_blocks_per_s": done * (tree_aes_per_launch(sub, b) + top) / dt}


def _round_key(path: str):
    """profiles/r14a_full_domain_summary.json -> (14, "a"): summaries sort by round."""
    m = re.match(r"r(\d+)([a-z]*)", os.path.basename(path))
    return (int(m.group(1)), m.group(2)) if m else (0, "")


def profiled_traffic(kernel: str, leaves_per_launch: int = None, workload: str = None):
    """Per-launch HBM bytes of the dominant kernel from the newest committed
    rocprofv3 PMC summary of this workload: profiles/<round>_<workload>_summary.json,
    written by tools/profile_workload.sh (tools/pmc_summary.py --workload) from
    the same bench.py command (FETCH_SIZE/WRITE_SIZE with the gfx950
    corrections of MI355X_MICROARCH.md).  Summaries without a workload tag
    (rounds before r14) are matched by kernel name (and outputs per launch)
    only when no tagged one exists."""
    tagged, untagged = [], []
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*_summary.json")):
        try:
            s = json.load(open(f))
        except (OSError, ValueError):
            continue
        if "hbm_traffic_bytes" not in s:
            continue
        if workload is not None and s.get("workload") == workload:
            tagged.append((_round_key(f), f, s))
        elif (s.get("workload") is None
              and kernel.replace("(anonymous namespace)::", "")
              in s.get("kernel", "").replace("(anonymous namespace)::", "")
              and (leaves_per_launch is None or s.get("leaves_per_launch") == leaves_per_launch)):
            untagged.append((_round_key(f), f, s))
    if not tagged and not untagged:
        return None
    _, f, s = max(tagged or untagged, key=lambda c: (c[0], c[1]))
    return (s["hbm_traffic_bytes"], os.path.relpath(f, ROOT),
            {"valu_lane_ops_per_aes": s.get("valu_lane_ops_per_aes"),
             "lds_lane_ops_per_aes": s.get("lds_lane_ops_per_aes"),
             "lds_pipe_busy": s.get("lds_pipe_busy"),
             "sustained_clock_ghz": s.get("effective_clock_ghz"),
             "clk_per_aes_per_cu": s.get("clk_per_aes_per_cu"),
             "write_amplification": s.get("write_amplification"),
             "hbm_write_bytes": s.get("hbm_write_bytes"),
             "hbm_read_bytes": s.get("hbm_read_bytes_corrected"),
             "profiled_kernel": s.get("kernel"),
             "profiled_launch_ms": s.get("avg_ns", 0) / 1e6})


def host_output_rate(dpf, ctx0, bits: int, reps: int, dev_out, n: int, kernel_ms: float) -> dict:
    """API-level throughput of the drop-in call the reference's callers make:
    EvaluateUntil<T>(0, {}, ctx) -> std::vector<T> in host memory
    (dpf/distributed_point_function.h:790-821), T = uint64_t / absl::uint128,
    on fresh copies of the benchmark key's context (C++ timing, GIL released).
    Its outputs are checked against the device run's at a few positions."""
    import statistics
    esz = bits // 8
    probe = [0, 1, n // 3, n // 2, n - 1]
    secs, got_n, samples = dpf._impl.time_evaluate_until(0, ctx0.SerializeToString(), bits, reps,
                                                          probe)
    assert got_n == n, (got_n, n)
    dev = dev_out.view(-1)
    for i, lo, hi in samples:
        b = dev[i * esz:(i + 1) * esz].cpu().numpy().tobytes()
        want = int.from_bytes(b, "little")
        assert (lo | hi << 64) == want, ("host vs device output", i)
    med = statistics.median(secs)
    nbytes = n * esz
    d2h_s = max(med - kernel_ms * 1e-3, 1e-9)
    return {"call": f"EvaluateUntil<{'uint64_t' if bits == 64 else 'absl::uint128'}>(0, {{}}, ctx) "
                    f"-> std::vector (host memory)",
            "reps": reps, "api_ms_per_call": [x * 1e3 for x in secs], "api_ms_per_step": med * 1e3,
            "api_leaves_per_s": n / med, "host_output_bytes": nbytes,
            "host_output_gb_per_s": nbytes / med / 1e9,
            "kernel_ms_per_step": kernel_ms,
            "d2h_gb_per_s_beyond_kernel": nbytes / d2h_s / 1e9,
            "note": "PCIe-inclusive; the kernel-level `value` keeps the outputs in HBM"}


def profile_check(roof: dict, tr, aes_per_launch: float, launch_ms: float) -> None:
    """Puts the committed rocprofv3 summary's timed-launch average beside this
    run's own HIP-event launch time: `frac_from_profile` is the roofline
    fraction the summary alone gives, `profile_vs_launch` their ratio (a
    summary of this kernel on this tree agrees within a few per cent)."""
    if not tr or not tr[2] or not tr[2].get("profiled_launch_ms"):
        return
    prof_ms = tr[2]["profiled_launch_ms"]
    roof["profiled_launch_ms"] = prof_ms
    roof["frac_from_profile"] = aes_per_launch / (prof_ms * 1e-3) / 1e9 / roof["peak"]
    roof["profile_vs_launch"] = prof_ms / launch_ms
    roof["profile_within_3pct"] = bool(abs(prof_ms / launch_ms - 1) <= 0.03)


def workload_tag(args) -> str:
    """The tools/profile_workload.sh tag of this bench workload (profiles/<round>_<tag>_summary.json)."""
    if args.workload == "full_domain_tuple":
        return f"full_domain_tuple_{args.tuple_type}"
    return args.workload


def kernel_name(args, bits: int) -> str:
    if args.workload == "full_domain_tuple":
        return ("expand_octet_kernel<Mod32Leaf<2> >" if args.tuple_type == "intmodn32x2"
                else "expand_octet_kernel<FastIntLeaf<32, false> >")
    return KERNEL.replace("64", str(bits))


def aes_rooflines(achieved: float, kernel: str, **extra) -> dict:
    """`roofline` against the integer-VALU AES roofline (north_star, SURVEY.md
    8d) and `roofline_lds` against the T-table's LDS bound, same achieved rate
    (algorithmic AES blocks per launch / HIP-event launch time)."""
    return {
        "roofline": {"bound": "valu", "achieved": achieved, "peak": AES_VALU_PEAK_GBLOCKS,
                     "unit": "G AES-128 blocks/s", "frac": achieved / AES_VALU_PEAK_GBLOCKS,
                     "kernel": kernel, **extra},
        "roofline_lds": {"bound": "lds", "achieved": achieved, "peak": AES_LDS_PEAK_GBLOCKS,
                         "unit": "G AES-128 blocks/s", "frac": achieved / AES_LDS_PEAK_GBLOCKS},
        "roofline_lds_measured": {"bound": "lds, measured lookup ceiling", "achieved": achieved,
                                  "peak": AES_LDS_MEASURED_GBLOCKS, "unit": "G AES-128 blocks/s",
                                  "frac": achieved / AES_LDS_MEASURED_GBLOCKS,
                                  "source": "profiles/r16/lds_ceiling.txt (2.4 GHz nominal)"},
    }


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(argv, n: int, port: int) -> list:
    """The torch.distributed.run command that runs this script as n ranks
    (one process per GPU, rendezvous on 127.0.0.1) with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
            "--master-port", str(port), os.path.abspath(__file__), *argv]


def maybe_self_launch(args, argv=None) -> None:
    """`python bench.py --gpus N` (N > 1) without a launcher: start the N ranks
    as child processes of a torch.distributed.run launcher, relay rank 0's
    JSON line, and exit with the launcher's status -- never fall back to one
    rank.  Runs before anything touches the GPU (torch.cuda.device_count()
    does not initialise HIP on this image; the children are started with
    subprocess, not exec).  Fewer visible devices than N is an error, except
    under DPF_BENCH_ONE_GPU=1 (every rank on cuda:0, the one-GPU rehearsal)."""
    if args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least one GPU")
    if args.workload.startswith("synthetic") and args.gpus != 1:
        raise SystemExit("synthetic_* workloads evaluate one key on one GPU (--gpus 1)")
    if "WORLD_SIZE" in os.environ:
        ws = int(os.environ["WORLD_SIZE"])
        if ws != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={ws}: the launcher started "
                             f"{ws} ranks")
        return
    if args.gpus == 1:
        return
    import subprocess
    import torch
    have = torch.cuda.device_count()
    need = 1 if os.environ.get("DPF_BENCH_ONE_GPU") == "1" else args.gpus
    if have < need:
        raise SystemExit(f"--gpus {args.gpus}: only {have} GPU(s) visible; refusing to run "
                         f"fewer ranks than asked")
    argv = sys.argv[1:] if argv is None else argv
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(launcher_cmd(argv, args.gpus, _free_port()), cwd=ROOT, env=env,
                            stdout=subprocess.PIPE, text=True)
    lines = 0
    for line in proc.stdout:           # rank 0's JSON line; anything else goes to stderr
        if line.startswith("{"):
            lines += 1
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
    rc = proc.wait()
    if rc == 0 and lines != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {lines}", file=sys.stderr)
        rc = 1
    raise SystemExit(rc)


def init_ranks(torch, dist, gpus: int = None):
    """One process per GPU (RANK/LOCAL_RANK/WORLD_SIZE from torch.distributed.run),
    RCCL process group for N > 1.  Returns (world, rank, local, coll), `coll`
    the device for collective scalars (None: host tensors).  `gpus` (the
    --gpus flag) must equal the launcher's world size.
    DPF_BENCH_ONE_GPU=1 rehearses the N-rank path on a one-GPU box: every rank
    on cuda:0, a gloo group (RCCL refuses two ranks on one device).
    DPF_BENCH_FORCE_PG=1 builds the RCCL group even for one rank, so every
    collective of the N-rank path (the max-over-ranks timing, the share
    all-reduce) runs through RCCL on a one-GPU box (tests/test_rccl_gpu.py)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if gpus is not None and world != gpus:
        raise SystemExit(f"--gpus {gpus} but {world} rank(s) running")
    one_gpu = os.environ.get("DPF_BENCH_ONE_GPU") == "1"
    force = os.environ.get("DPF_BENCH_FORCE_PG") == "1"
    if one_gpu:
        local = 0
    coll = None
    if world > 1 or force:
        torch.cuda.set_device(local)
        if world == 1:        # a one-rank group outside a launcher
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if one_gpu and world > 1:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            coll = torch.device("cuda", local)
    return world, rank, local, coll


def group_up(dist) -> bool:
    """A process group exists (N > 1, or one forced rank)."""
    return dist.is_available() and dist.is_initialized()


def main():
    args = parse()
    maybe_self_launch(args)
    if args.workload.startswith("evaluate_at"):
        return main_evaluate_at(args)
    if args.workload.startswith("synthetic"):
        return main_synthetic(args)
    if args.workload == "heavy_hitters":
        return main_heavy_hitters(args)
    if args.workload == "dcf":
        return main_dcf(args)
    if args.workload == "full_domain_u128" and args.log_domain == LOG_PER_GPU:
        args.log_domain = 31
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import hip_abi as H
    from distributed_point_functions_amd import proto as pb
    from distributed_point_functions_amd import sharding as S

    world, rank, local, coll = init_ranks(torch, dist, args.gpus)
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)

    bits = 128 if args.workload == "full_domain_u128" else 64
    esz = bits // 8
    # The partition: `shards` subtrees of which this process evaluates shard
    # `shard` (rank r of N; shard 0 of W in a --rehearse-world W run).
    shards, shard = (args.rehearse_world, 0) if args.rehearse_world else (world, rank)
    log_domain = (S.weak_scaling_log_domain(args.log_domain, shards) if args.scaling == "weak"
                  else args.log_domain)
    params = pb.DpfParameters()
    params.log_domain_size = log_domain
    if args.workload == "full_domain_tuple":
        # Tuple leaves: both types pack to 8 bytes.
        if args.tuple_type == "intmodn32x2":
            el = D.int_mod_n_type(32, 4294967291)
            vtype, beta_py = D.tuple_type(el, el), (123456789, 4000000000)
        else:
            vtype, beta_py = D.tuple_type(D.integer_type(32), D.integer_type(32)), (0xDEADBEEF, 7)
    else:
        vtype, beta_py = D.integer_type(bits), 0xDEADBEEF
    params.value_type.CopyFrom(vtype)
    dpf = D.DistributedPointFunction.create(params)
    if args.workload == "full_domain_tuple":
        dpf.register_value_type(vtype)
    # Same key on every rank: root seeds injected (GenerateKeysIncrementalWithSeeds).
    alpha = 0x2545F4914F6CDD1D % (1 << log_domain)
    beta = D.to_value(vtype, beta_py)
    key, _ = dpf.generate_keys_incremental(alpha, [beta], seeds=(0x243F6A8885A308D3,
                                                                 0x13198A2E03707344))
    ctx0 = dpf.create_evaluation_context(key)
    depth = dpf.hierarchy_to_tree()[0] - S.shard_bits(shards)   # tree levels expanded per rank
    outputs_per_rank = 1 << S.strong_scaling_log_outputs(log_domain, shards)
    out = torch.empty(outputs_per_rank * esz, dtype=torch.uint8, device=dev)

    def step(evs=None):
        ctx = pb.EvaluationContext()
        ctx.CopyFrom(ctx0)
        if evs is not None:
            evs[0].record(stream)
        n = dpf.evaluate_shard_to_device(0, shard, shards, ctx, out, stream=stream)
        if evs is not None:
            evs[1].record(stream)
        return n

    for _ in range(args.warmup):
        assert step() == outputs_per_rank
    torch.cuda.synchronize(dev)
    if group_up(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(H.Event(), H.Event()) for _ in range(args.steps)]
    H.clock_probe(True)          # two s_memtime/s_memrealtime stamps per workgroup
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    clock = H.clock_probe_read()
    H.clock_probe(False)
    if group_up(dist):
        dist.barrier()
    per_step_ms = [a.elapsed_ms(b) for a, b in evs]
    kern_ms = float(np.mean(per_step_ms))
    elapsed = S.max_over_ranks(t1 - t0, device=coll)
    kern_ms_max = S.max_over_ranks(kern_ms, device=coll)
    ginfo = S.group_info(kern_ms, device=coll)
    clocks = S.gather_over_ranks(clock["clock_ghz"], device=coll)

    # Spot-check the last step's output (sum of the two parties' shares is beta
    # at alpha, 0 elsewhere) on a few positions of this rank's shard.
    _check_shard(dpf, key, out, shard, shards, outputs_per_rank, alpha, bits)

    # Value hashes per leaf: the blocks the conversion reads (b = 1 for
    # integers and direct tuples; 2 for Tuple<IntModN32 x 2>: 16 + 4 bytes
    # sampled, value_type_helpers.h:415-443).  The reference hashes
    # blocks_needed blocks per leaf (HashExpandedSeeds, cc:500-524).
    tuple_mod = args.workload == "full_domain_tuple" and args.tuple_type == "intmodn32x2"
    b_read = 2 if tuple_mod else 1
    aes_per_launch = tree_aes_per_launch(depth, b_read)
    ref_aes_per_launch = tree_aes_per_launch(depth, dpf.blocks_needed(0))
    achieved = aes_per_launch / (kern_ms_max * 1e-3) / 1e9
    bytes_per_launch = outputs_per_rank * esz
    ms_per_step = elapsed * 1e3 / args.steps
    total = outputs_per_rank * world * args.steps
    n_cus = torch.cuda.get_device_properties(dev).multi_processor_count
    # 0 workgroups stamped: the launches ran a kernel without the probe
    # (expand_small_kernel, latency mode: config 1) -- no clock, not 0 GHz.
    ghz = clock["clock_ghz"] if clock["workgroups"] else None
    if rank == 0:
        # The committed rocprof summaries are of the one-GPU lines.
        tr = (profiled_traffic(kernel_name(args, bits), outputs_per_rank, workload=workload_tag(args))
              if shards == 1 and args.log_domain == (31 if bits == 128 else LOG_PER_GPU) else None)
        vname = {"full_domain": "uint64", "full_domain_u128": "uint128",
                 "full_domain_tuple": {"intmodn32x2": "Tuple<IntModN<uint32_t, 4294967291>, "
                                                      "IntModN<uint32_t, 4294967291>>",
                                       "u32x2": "Tuple<uint32_t, uint32_t>"}[args.tuple_type]
                 }[args.workload]
        res = {
            "metric": METRIC if args.workload == "full_domain" else
                      f"DPF leaf evals/sec, full-domain {vname}; AES blocks/s",
            "value": total / elapsed,
            "unit": "leaves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u32 mod N" if tuple_mod else ("u32" if args.workload == "full_domain_tuple"
                                                   else f"u{bits}"),
            "data": "synthetic: one DpfKey from the product keygen with fixed root seeds",
            "reference_aes_blocks_per_launch": ref_aes_per_launch,
            "config": {"workload": f"full-domain EvaluateUntil(0, {{}}) of one key, "
                                   f"log_domain_size={log_domain}, {vname}, "
                                   f"2^{outputs_per_rank.bit_length() - 1} outputs per GPU",
                       "log_domain_size": log_domain, "value_type": vname,
                       "blocks_needed": dpf.blocks_needed(0), "value_blocks_hashed_per_leaf": b_read,
                       "outputs_per_gpu": outputs_per_rank, "tree_levels_per_gpu": depth,
                       "parallelism": f"subtree-prefix x{shards}"},
            "aes_blocks_per_s": aes_per_launch * world * args.steps / elapsed,
            **aes_rooflines(achieved, kernel_name(args, bits),
                            traffic=tr[0] if tr else None,
                            traffic_source=tr[1] if tr else None,
                            pmc=tr[2] if tr else None, launch_ms=kern_ms_max,
                            algorithmic_aes_per_launch=aes_per_launch,
                            algorithmic_bytes_per_launch=bytes_per_launch,
                            sustained_clock_ghz=ghz,
                            sustained_clock_ghz_per_rank=clocks,
                            clk_per_aes_per_cu=(kern_ms * 1e-3 * ghz * 1e9 * n_cus / aes_per_launch
                                                if ghz else None),
                            clock_source=("s_memtime/s_memrealtime stamps of every workgroup of the "
                                          f"timed launches ({clock['workgroups']} workgroups, "
                                          f"{clock['mean_workgroup_ms']:.3f} ms each on average)"
                                          if ghz else "none: the timed kernel carries no clock probe"),
                            cus=n_cus),
            # Fixed per-step cost: wall time per step beyond the launch's own
            # HIP-event time (host validation, the packed image, launch gaps).
            "step_overhead": {"ms_per_step": ms_per_step, "launch_ms": kern_ms_max,
                              "overhead_ms": ms_per_step - kern_ms_max,
                              "overhead_frac": (ms_per_step - kern_ms_max) / ms_per_step,
                              # rank 0's launches in order: a clock still ramping
                              # shows as first >> last.
                              "launch_ms_first": per_step_ms[0], "launch_ms_last": per_step_ms[-1],
                              "launch_ms_min": min(per_step_ms), "launch_ms_max": max(per_step_ms)},
            "process_group": ginfo,
            "roofline_hbm": {"bound": "hbm",
                             "achieved": bytes_per_launch / (kern_ms_max * 1e-3) / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": bytes_per_launch / (kern_ms_max * 1e-3) / 1e9 / HBM_PEAK_GBS},
        }
        if args.rehearse_world:
            res["rehearsal"] = (f"one process evaluating shard 0 of a {shards}-rank split: "
                                f"`value` is that shard's rate on one GPU, not an N-GPU result")
        profile_check(res["roofline"], tr, aes_per_launch, kern_ms_max)
        if (args.host_output and world == 1 and shards == 1
                and args.workload in ("full_domain", "full_domain_u128")):
            res["api_level"] = host_output_rate(dpf, ctx0, bits, args.host_output_reps, out,
                                                outputs_per_rank, kern_ms_max)
        if world == 1 and not args.no_cpu_baseline:
            ovt = None
            if args.workload == "full_domain_tuple":
                ovt = (("tuple", [("intmodn", 32, 4294967291)] * 2)
                       if args.tuple_type == "intmodn32x2" else ("tuple", [("int", 32)] * 2))
            res["cpu_baseline"] = cpu_baseline(key, log_domain, args.cpu_chunks, bits, vt=ovt)
        print(json.dumps(res), flush=True)
    if group_up(dist):
        dist.destroy_process_group()


EA_METRIC = ("batched EvaluateAt point evals/sec, 2^20 keys x 2^10 points each, log_domain 128, "
             "uint64 (BASELINE configs[3]); AES blocks/s")
EA_SUM_METRIC = ("aggregated EvaluateAt point evals/sec (sum over 2^20 keys at 2^10 shared points), "
                 "log_domain 128, uint64 (BASELINE configs[3] aggregation variant)")


def _oracle_key(key):
    """A product DpfKey proto restated as the oracle's key dict (single level)."""
    return {"seed": key.seed.high << 64 | key.seed.low, "party": key.party,
            "cws": [(c.seed.high << 64 | c.seed.low, int(c.control_left), int(c.control_right),
                     None) for c in key.correction_words],
            "last_vc": [_leaf_ints(v) for v in key.last_level_value_correction]}


def cpu_baseline_points(dpf, batch, host_points, keys: int, ppk: int):
    """The reference's EvaluateAt CPU path (EvaluateAtImpl, distributed_point_
    function.h:839-1010, with the Highway one-AES-per-level EvaluateSeeds,
    evaluate_prg_hwy.cc:205-304) restated on AES-NI (oracle/cpu_baseline.c, 8
    points interleaved per thread; tests/test_oracle.py checks it equals the
    oracle) on a bounded sample of the workload: the first keys of the batch x
    their ppk points, chunks of 32 keys spread over baseline_threads() host
    threads for ~15 s, plus a 3 s single-thread sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nk = min(keys, 32768)
    protos = [dpf.key_from_batch(batch, k) for k in range(nk)]
    L = len(protos[0].correction_words) - 1          # 127 tree levels below the root
    seeds = np.array([[p.seed.low, p.seed.high] for p in protos], np.uint64)
    party = np.array([p.party for p in protos], np.uint8)
    cws = np.array([[[c.seed.low, c.seed.high] for c in p.correction_words[:L]] for p in protos],
                   np.uint64)
    cl = np.array([[c.control_left for c in p.correction_words[:L]] for p in protos], np.uint8)
    cr = np.array([[c.control_right for c in p.correction_words[:L]] for p in protos], np.uint8)
    vcw = np.array([[[_int_of(v) & (2**64 - 1), 0] for v in p.last_level_value_correction]
                    for p in protos], np.uint64)
    pts = np.ascontiguousarray(host_points[:nk * ppk].reshape(nk, ppk, 2))
    chunk = 32

    def work(c):
        sl = slice(c * chunk, min(nk, (c + 1) * chunk))
        O.baseline_evaluate_at_u64(L, 1, seeds[sl], party[sl], cws[sl], cl[sl], cr[sl], vcw[sl],
                                   pts[sl])
        return (sl.stop - sl.start) * ppk

    T = baseline_threads()
    n, dt, done = run_cpu_pool(work, range((nk + chunk - 1) // chunk), threads=T, budget_s=15.0)
    n1, dt1, done1 = run_cpu_pool(work, range((nk + chunk - 1) // chunk), threads=1, budget_s=3.0)
    return {"value": n / dt, "unit": "points/s", "cores": T, "kind": "port", "host": host_cpu(T),
            "single_thread_value": n1 / dt1,
            "all_cores": all_cores_sample(work, range((nk + chunk - 1) // chunk), "points/s"),
            "published_reference_single_thread": "335K points/s (2^20 points at log 128 in "
                                                 "3.13 s, experiments/README.md:98-107, one "
                                                 "Xeon thread @ 2.3 GHz)",
            "sample": f"{done * chunk} keys x {ppk} points of the benchmark batch (log 128, "
                      f"uint64): the reference's one-AES-per-level path walk + value hash + "
                      f"correction on AES-NI (oracle/cpu_baseline.c); {dt:.1f} s wall on {T} "
                      f"host threads",
            "aes_blocks_per_s": n * 128 / dt}


def main_evaluate_at(args):
    """EvaluateAt for 2^20 keys x 2^10 points on a 2^128
    domain (uint64), keys split across ranks (DeviceKeyBatch rows [lo, hi)).
    `evaluate_at`: independent points per key, outputs [key][point] stay in HBM.
    `evaluate_at_sum`: one shared point set, sum over keys on the device, then
    the per-rank partial sums are all-gathered (RCCL) and group-summed."""
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import hip_abi as H
    from distributed_point_functions_amd import proto as pb
    from distributed_point_functions_amd import sharding as S

    world, rank, local, coll = init_ranks(torch, dist, args.gpus)
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    summed = args.workload == "evaluate_at_sum"

    params = pb.DpfParameters()
    params.log_domain_size = 128
    params.value_type.CopyFrom(D.integer_type(64))
    dpf = D.DistributedPointFunction.create(params)
    n_keys, ppk = 1 << args.keys_log, 1 << args.points_log
    lo, hi = S.key_range(n_keys, world, rank)
    nk = hi - lo
    # Keys: seeded alphas and root seeds for ALL keys (identical whatever the
    # world size); each rank generates and uploads only its rows.
    rng = np.random.default_rng(0xC0F4)
    alphas = rng.integers(0, 2**64, size=(n_keys, 2), dtype=np.uint64)
    seeds = rng.integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    beta = D.to_value(D.integer_type(64), 1)
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    b0, b1 = dpf.generate_key_batch(alphas[lo:hi], [beta], root_seeds=seeds[2 * lo:2 * hi],
                                    threads=threads)
    keygen_s = time.perf_counter() - t0
    # Key ingestion: the rank's keys as serialized DpfKeys
    # (the reference's wire format), parsed into the SoA batch on host threads
    # and uploaded -- the path a server receiving client keys takes.
    t0 = time.perf_counter()
    wire = dpf.serialize_key_batch(b0, threads=threads)
    serialize_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    parsed = dpf.parse_key_batch(wire, threads=threads)
    parse_s = time.perf_counter() - t0
    if not np.array_equal(parsed.seeds(), b0.seeds()):
        raise SystemExit("parsed key batch differs from the generated one")
    ingest = {"keys": nk, "wire_bytes": sum(len(w) for w in wire), "threads": threads,
              "serialize_s": serialize_s, "parse_s": parse_s, "parse_keys_per_s": nk / parse_s}
    del wire
    t0 = time.perf_counter()
    dbatch = dpf.upload_key_batch(parsed, stream=stream)
    torch.cuda.synchronize(dev)
    ingest["upload_s"] = time.perf_counter() - t0
    del parsed
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    if summed:
        shared = rng.integers(0, 2**64, size=(ppk, 2), dtype=np.uint64)
        shared[:4] = alphas[:4]          # four points hit one client each (reconstruction check)
        points = torch.from_numpy(shared.view(np.int64)).to(dev)
        out = torch.empty(ppk * 8, dtype=torch.uint8, device=dev)
    else:
        points = torch.randint(-2**63, 2**63 - 1, (nk * ppk, 2), dtype=torch.int64, device=dev,
                               generator=gen)
        out = torch.empty(nk * ppk * 8, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        if summed:
            dpf.evaluate_at_batch_sum_to_device(dbatch, 0, points, out, stream=stream)
        else:
            dpf.evaluate_at_batch_to_device(dbatch, 0, points, ppk, out, stream=stream)
        if evs is not None:
            evs[1].record(stream)
        if summed and group_up(dist):
            return S.aggregate_shares(dpf, 0, out, ppk)
        return None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if group_up(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(H.Event(), H.Event()) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        total = step(evs[i])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    timed_kernel = H.last_points_kernel()   # before the spot checks launch their own
    if group_up(dist):
        dist.barrier()
    kern_ms = float(np.mean([a.elapsed_ms(b) for a, b in evs]))
    elapsed = S.max_over_ranks(t1 - t0, device=coll)
    kern_ms_max = S.max_over_ranks(kern_ms, device=coll)
    ginfo = S.group_info(kern_ms, device=coll)

    # Correctness spot checks outside the timed region.
    if summed:
        s0 = total if total is not None else out.cpu().numpy()
        dpf.evaluate_at_batch_sum_to_device(dpf.upload_key_batch(b1, stream=stream), 0, points,
                                            out, stream=stream)
        s1 = S.aggregate_shares(dpf, 0, out, ppk) if group_up(dist) else out.cpu().numpy()
        rec = (np.asarray(s0).view(np.uint64) + np.asarray(s1).view(np.uint64)).tolist()
        if rec != [1, 1, 1, 1] + [0] * (ppk - 4):
            raise SystemExit(f"rank {rank}: two-server reconstruction failed: {rec[:8]}")
    else:
        host_pts = points.view(-1, 2)
        for k in (0, nk // 2, nk - 1):
            pk = host_pts[k * ppk:(k + 1) * ppk].cpu().numpy().view(np.uint64)
            pts = [int(a) | int(b) << 64 for a, b in pk[:64]]
            want = dpf.evaluate_at(dpf.key_from_batch(b0, k), 0, pts)
            got = out.view(torch.int64)[k * ppk:k * ppk + 64].cpu().numpy().view(np.uint64)
            if not np.array_equal(got, want):
                raise SystemExit(f"rank {rank}: batch output of key {lo + k} disagrees with EvaluateAt")

    depth = dpf.hierarchy_to_tree()[0]                 # 127 path levels, + 1 value hash
    aes_per_launch = nk * ppk * (depth + 1)
    achieved = aes_per_launch / (kern_ms_max * 1e-3) / 1e9
    # The point kernel the timed launches ran (dpf_hip_last_points_kernel):
    # four path chains per lane at this size, two otherwise.
    if timed_kernel == "points/ilp4":
        kname = "eval_points4_kernel<64, true, %s>" % ("true" if summed else "false")
    else:
        kname = ("eval_points_kernel<(anonymous namespace)::GenericLeaf, 64, true, true, %s" %
                 ("true>" if summed else "false, true>"))
    tr = (profiled_traffic(kname, workload=args.workload)
          if n_keys == 1 << 20 and ppk == 1 << 10 and world == 1 else None)
    if rank == 0:
        res = {
            "metric": EA_SUM_METRIC if summed else EA_METRIC,
            "value": n_keys * ppk * args.steps / elapsed,
            "unit": "points/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: 2^20 key pairs from the product batched keygen (seeded alphas and "
                    "root seeds, beta = 1), uniform random 128-bit points",
            "config": {"workload": ("EvaluateAt summed over keys at shared points" if summed else
                                    "EvaluateAt, independent points per key") +
                                   f", {n_keys} keys x {ppk} points, log_domain_size=128, uint64",
                       "keys": n_keys, "points_per_key": ppk, "log_domain_size": 128,
                       "parallelism": f"key-batch x{world}"},
            "aes_blocks_per_s": n_keys * ppk * (depth + 1) * args.steps / elapsed,
            "keygen_s_rank0": keygen_s, "keygen_threads": threads, "key_ingest_rank0": ingest,
            **aes_rooflines(achieved, kname, traffic=tr[0] if tr else None,
                            traffic_source=tr[1] if tr else None, pmc=tr[2] if tr else None,
                            launch_ms=kern_ms_max, algorithmic_aes_per_launch=aes_per_launch),
            "process_group": ginfo,
        }
        profile_check(res["roofline"], tr, aes_per_launch, kern_ms_max)
        if world == 1 and not args.no_cpu_baseline:
            nb = min(nk, 32768)
            if summed:
                host_pts = np.tile(shared.astype(np.uint64), (nb, 1))
            else:
                host_pts = points.view(-1, 2)[:nb * ppk].cpu().numpy().view(np.uint64)
            res["cpu_baseline"] = cpu_baseline_points(dpf, b0, host_pts, nk, ppk)
        print(json.dumps(res), flush=True)
    if group_up(dist):
        dist.destroy_process_group()


# experiments/README.md (1 key, 2^20 nonzeros, uint32, one Xeon thread @ 2.30 GHz):
# seconds per iteration by (mode, domain, distribution).
PUBLISHED_SYNTHETIC = {
    ("hierarchical", 32): {"0.1": 1.36, "0.5": 2.22, "uniform": 3.31},
    ("direct", 32): {"0.1": 0.67, "0.5": 0.68, "uniform": 0.70},
    ("hierarchical", 128): {"0.1": 32.68, "0.5": 35.07, "uniform": 35.95},
    ("direct", 128): {"0.1": 3.08, "0.5": 3.13, "uniform": 3.13},
}


def main_synthetic(args):
    """the reference's own published benchmark
    (experiments/synthetic_data_benchmarks.cc) -- one key, 2^20 nonzeros,
    uint32, hierarchical EvaluateUntil over levels chosen so no level expands to
    more than 4 x 2^20 outputs, or direct EvaluateAt at the nonzeros -- run
    through the same driver restated in C++ on the GPU-backed API.  The
    reference's CSV inputs are git-LFS stubs; the nonzeros are regenerated
    with the README's distributions (seeded).  Single key => one GPU."""
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import hip_abi as H
    if int(os.environ.get("WORLD_SIZE", "1")) != 1 or args.gpus != 1:
        raise SystemExit("synthetic_* workloads evaluate one key on one GPU (--gpus 1)")
    H.load(require_gpu=True)
    mode = "direct" if args.workload == "synthetic_direct" else "hierarchical"
    device_ctx = args.workload == "synthetic_hierarchical_device"
    conc = 0.0 if args.distribution == "uniform" else float(args.distribution)
    host = D.host()
    # warmup iteration(s) are part of the driver's first call; time a second call.
    for _ in range(max(args.warmup, 0)):
        D._call(host.run_synthetic_data_benchmark, args.domain, 1 << 20, conc, 1, 4, 1,
                mode == "direct", False, device_ctx)
    r = D._call(host.run_synthetic_data_benchmark, args.domain, 1 << 20, conc, 1, 4,
                args.steps, mode == "direct", True, device_ctx)
    pub = PUBLISHED_SYNTHETIC.get((mode, args.domain), {}).get(args.distribution)
    secs = r["seconds_per_iteration"]
    outs = sum(r["outputs_per_level"])
    res = {
        "metric": f"synthetic_data_benchmarks {mode} evaluation, domain 2^{args.domain}, "
                  f"distribution {args.distribution}: seconds per iteration (1 key, 2^20 nonzeros, uint32)",
        "value": secs, "unit": "s/iteration", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": secs * 1e3, "higher_is_better": False,
        "scaling": "none", "vs_baseline": (secs / pub) if pub else None,
        "published_reference_s": pub, "dtype": "u32",
        "data": "synthetic: 2^20 distinct nonzeros regenerated with the README's distributions "
                "(the reference CSVs are git-LFS stubs); seed 1",
        "config": {"workload": f"{mode} evaluation of one DpfKey through the DistributedPointFunction "
                               f"API (EvaluateUntil per level / EvaluateAt), domain 2^{args.domain}" +
                               (", device-resident context (EvaluateUntilBatchToDevice on a one-key "
                                "batch, outputs copied to host per level)" if device_ctx else ""),
                   "levels_to_evaluate": r["levels_to_evaluate"],
                   "prefixes_per_level": r["prefixes_per_level"],
                   "outputs_per_level": r["outputs_per_level"],
                   "key_size_bytes": r["key_size_bytes"]},
        "outputs_per_s": outs / secs, "verified_two_server_reconstruction": r["verified"],
        # This build's XOR-fold of every output (its cross-check of the device
        # context against EvaluateUntil's outputs) runs inside the iterations
        # but is not the reference's work (synthetic_data_benchmarks.cc:169-191
        # only returns the outputs): timed apart and excluded from `value`.
        "checksum_seconds_excluded": r.get("checksum_seconds_excluded"),
    }
    print(json.dumps(res), flush=True)


HH_METRIC = ("heavy-hitters prefix evals/sec: 2^20 clients, 128-bit hierarchy {8,10,...,128}, "
             "Tuple<IntModN32,IntModN32>, top-1024 candidates per level, both servers")


def main_heavy_hitters(args):
    """2^20 client keys per server, 61-level 128-bit
    hierarchy, per level EvaluateUntil of every key at the <= 1024 current
    candidates x 4 children, summed over keys on the device (device-resident
    batch context), per-rank sums all-gathered (RCCL) and group-summed, the
    two servers' sums added and the next candidates selected.  One step = one
    full pass over all levels for BOTH servers; clients are split across ranks
    (strong scaling)."""
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import heavy_hitters as HH
    from distributed_point_functions_amd import hip_abi as H
    from distributed_point_functions_amd import sharding as S

    world, rank, local, coll = init_ranks(torch, dist, args.gpus)
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)

    logs = HH.hierarchy()
    dpf = HH.create_dpf(logs)
    n_keys = 1 << args.keys_log
    values, idx, alphas = HH.client_values(n_keys, seed=0x5B)
    lo, hi = S.key_range(n_keys, world, rank)
    rng = np.random.default_rng(0x5B5B)
    seeds = rng.integers(0, 2**64, size=(2 * n_keys, 2), dtype=np.uint64)
    beta = D.to_value(HH.value_type(), HH.BETA)
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    b0, b1 = dpf.generate_key_batch(alphas[lo:hi], [beta] * len(logs),
                                    root_seeds=seeds[2 * lo:2 * hi], threads=threads)
    keygen_s = time.perf_counter() - t0
    max_out = max(4 * args.top_k, 1 << logs[0])
    servers = [HH.Server(dpf, dpf.upload_key_batch(b, stream=stream), max_out, dev)
               for b in (b0, b1)]
    aggregate = ((lambda h, part, n: S.aggregate_shares(dpf, h, part, n)) if group_up(dist)
                 else None)
    evs = []

    class Timed:  # brackets every batched evaluation with hipEvents on `stream`
        def __init__(self, srv):
            self.srv, self.out = srv, srv.out

        def evaluate(self, level, prefixes, stream=None):
            a, b = H.Event(), H.Event()
            a.record(stream)
            n = self.srv.evaluate(level, prefixes, stream)
            b.record(stream)
            evs.append((a, b))
            return n

    def one_pass(record=None):
        for srv in servers:
            srv.reset()
        return HH.run(dpf, [Timed(s) for s in servers], logs, args.top_k, aggregate, stream,
                      record, keep_cache=True)

    for _ in range(args.warmup):
        one_pass()
    torch.cuda.synchronize(dev)
    if group_up(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs.clear()
    record = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        final = one_pass(record if i == args.steps - 1 else None)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if group_up(dist):
        dist.barrier()
    kern_ms = sum(a.elapsed_ms(b) for a, b in evs) / args.steps
    cache_bytes = [int(srv.ctx.device_bytes) for srv in servers]
    for srv in servers:           # kept across the passes, given back now
        srv.release_expansion_cache()
    elapsed = S.max_over_ranks(t1 - t0, device=coll)
    kern_ms_max = S.max_over_ranks(kern_ms, device=coll)
    ginfo = S.group_info(kern_ms, device=coll)
    verified = os.environ.get("DPF_BENCH_SKIP_VERIFY") != "1"  # probe libraries only
    if rank == 0 and verified:
        HH.verify(record, logs, values, idx)        # every level, untimed
    outputs_per_pass = sum(len(v) for _, v, _, _ in record) * n_keys * 2
    # The device contexts' expansion cache (default; DPF_BATCH_NO_CACHE=1 turns
    # it off) spares the path steps: only AES actually computed are counted.
    cache = os.environ.get("DPF_BATCH_NO_CACHE") != "1"
    aes_rank = HH.algorithmic_aes(dpf, logs, record, hi - lo, walk=not cache) * 2
    aes_total = HH.algorithmic_aes(dpf, logs, record, n_keys, walk=not cache) * 2
    achieved = aes_rank / (kern_ms_max * 1e-3) / 1e9
    tr = (profiled_traffic("batch_level_kernel<(anonymous namespace)::Mod32V<2, true>, 2, true>",
                           workload="heavy_hitters")
          if n_keys == 1 << 20 and world == 1 and args.top_k == 1024 else None)
    if rank == 0:
        ref = HH.plaintext_prefix_counts(values, idx, 128)
        true_top = set(sorted(ref, key=lambda v: (-ref[v], v))[:args.top_k])
        res = {
            "metric": HH_METRIC,
            "value": outputs_per_pass * args.steps / elapsed,
            "unit": "prefix evals/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u32 mod N",
            "data": "synthetic: 2^20 clients, values Zipf(1.1) over 2^14 random 128-bit values, "
                    "key pairs from the product batched keygen (seeded), beta = (1, 7)",
            "config": {"workload": f"heavy hitters, {n_keys} clients, {len(logs)} levels "
                                   f"(log {logs[0]}..{logs[-1]} step 2), top-{args.top_k}, "
                                   "EvaluateUntilBatchSumToDevice per level and server",
                       "keys": n_keys, "levels": len(logs), "top_k": args.top_k,
                       "parallelism": f"key-batch x{world}"},
            "seconds_per_pass": elapsed / args.steps,
            "expansion_cache": cache,
            "expansion_cache_events": [dict(srv.ctx.cache_events) for srv in servers],
            "batch_context_device_bytes": cache_bytes,
            "outputs_per_pass": outputs_per_pass,
            "aes_blocks_per_s": aes_total * args.steps / elapsed,
            "keygen_s_rank0": keygen_s, "keygen_threads": threads,
            "verified": ("two-server reconstruction == plaintext prefix histogram at every level"
                         if verified else False),
            "true_top_k_recall": len(true_top & set(final)) / max(len(true_top), 1),
            **aes_rooflines(achieved, "hh_keys_kernel (cached levels) + batch_level_kernel<Mod32V, 2, true> (level 0)",
                            traffic=tr[0] if tr else None, traffic_unit="bytes per pass",
                            traffic_source=tr[1] if tr else None, pmc=tr[2] if tr else None,
                            launch_ms_per_pass=kern_ms_max, algorithmic_aes_per_pass=aes_rank),
            "process_group": ginfo,
        }
        profile_check(res["roofline"], tr, aes_rank, kern_ms_max)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline_heavy_hitters(logs, record, alphas, seeds,
                                                             args.top_k)
        print(json.dumps(res), flush=True)
    if group_up(dist):
        dist.destroy_process_group()


DCF_METRIC = "batched DCF evals/sec (DistributedComparisonFunction::Evaluate), uint64, log domain 64"


def main_dcf(args):
    """DistributedComparisonFunction::Evaluate for K keys x
    2^points_log independent points each (uint64, log domain 64), keys split
    across ranks, outputs [key][point] in HBM.  One fused walk per (key, x)."""
    import torch
    import torch.distributed as dist
    from distributed_point_functions_amd import dcf as C
    from distributed_point_functions_amd import dpf as D
    from distributed_point_functions_amd import hip_abi as H
    from distributed_point_functions_amd import proto as pb
    from distributed_point_functions_amd import sharding as S

    world, rank, local, coll = init_ranks(torch, dist, args.gpus)
    H.load(require_gpu=True)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    n = args.dcf_log_domain
    params = pb.DcfParameters()
    params.parameters.log_domain_size = n
    params.parameters.value_type.CopyFrom(D.integer_type(64))
    dcf = C.DistributedComparisonFunction.create(params)
    n_keys, ppk = 1 << args.dcf_keys_log, 1 << args.points_log
    lo, hi = S.key_range(n_keys, world, rank)
    rng = np.random.default_rng(0xDCF)
    alphas = rng.integers(0, 2**63, size=n_keys, dtype=np.uint64)
    t0 = time.perf_counter()
    keys = [dcf.generate_keys(int(alphas[k]), 1, seed_0=2 * k + 1, seed_1=2 * k + 2)[0]
            for k in range(lo, hi)]
    keygen_s = time.perf_counter() - t0
    batch = dcf.make_key_batch(keys)
    dbatch = dcf.upload_key_batch(batch, stream=stream)
    gen = torch.Generator(device=dev)
    gen.manual_seed(99 + rank)
    nk = hi - lo
    pts = torch.randint(0, 2**63 - 1, (nk * ppk, 2), dtype=torch.int64, device=dev, generator=gen)
    if n <= 64:
        pts[:, 1] = 0
        if n < 64:
            pts[:, 0] &= (1 << n) - 1
    out = torch.empty(nk * ppk * 8, dtype=torch.uint8, device=dev)

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        dcf.evaluate_batch_to_device(dbatch, pts, ppk, out, stream=stream)
        if evs is not None:
            evs[1].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if group_up(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    evs = [(H.Event(), H.Event()) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if group_up(dist):
        dist.barrier()
    kern_ms = float(np.mean([a.elapsed_ms(b) for a, b in evs]))
    elapsed = S.max_over_ranks(t1 - t0, device=coll)
    kern_ms_max = S.max_over_ranks(kern_ms, device=coll)
    ginfo = S.group_info(kern_ms, device=coll)
    # Spot check against the single-key API (itself parity-tested vs the oracle).
    host_pts = pts.cpu().numpy().view(np.uint64)
    for k in (0, nk - 1):
        xs = [int(a) | int(b) << 64 for a, b in host_pts[k * ppk:k * ppk + 16]]
        want = dcf.evaluate_packed(keys[k], xs).view(np.uint64).reshape(-1)
        got = out.view(torch.int64)[k * ppk:k * ppk + 16].cpu().numpy().view(np.uint64)
        if not np.array_equal(got, want):
            raise SystemExit(f"rank {rank}: DCF batch output of key {lo + k} disagrees")
    h2t = dcf._impl.hierarchy_to_tree()
    aes_per_eval = h2t[-1] + (h2t[-1] + 1)      # walk + one value hash per depth
    aes_launch = nk * ppk * aes_per_eval
    achieved = aes_launch / (kern_ms_max * 1e-3) / 1e9
    tr = (profiled_traffic("dcf_fast_kernel<64, false, true, 1>", workload="dcf")
          if (n_keys, ppk, n, world) == (1 << 16, 1 << 10, 64, 1) else None)
    if rank == 0:
        res = {
            "metric": DCF_METRIC, "value": n_keys * ppk * args.steps / elapsed, "unit": "evals/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic: DCF keys from the product keygen (seeded), beta = 1, "
                    "uniform random points",
            "config": {"workload": f"DCF Evaluate, {n_keys} keys x {ppk} points, log domain {n}, "
                                   "uint64", "keys": n_keys, "points_per_key": ppk,
                       "log_domain_size": n, "parallelism": f"key-batch x{world}"},
            "aes_blocks_per_s": n_keys * ppk * aes_per_eval * args.steps / elapsed,
            "keygen_s_rank0": keygen_s,
            **aes_rooflines(achieved, "dcf_fast_kernel<64, false, true, 1>", traffic=tr[0] if tr else None,
                            traffic_source=tr[1] if tr else None, pmc=tr[2] if tr else None,
                            launch_ms=kern_ms_max, algorithmic_aes_per_launch=aes_launch),
            "process_group": ginfo,
        }
        profile_check(res["roofline"], tr, aes_launch, kern_ms_max)
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            P = O.dcf_params(n, ("int", 64))

            def work(i):
                ok = O.dcf_generate_keys(P, int(alphas[lo + i]), [1], 2 * i + 1, 2 * i + 2)[0]
                xs = [int(a) | int(b) << 64 for a, b in host_pts[i * ppk:i * ppk + 64]]
                for x in xs:
                    O.dcf_evaluate(P, ok, x)
                return len(xs)

            evals, dt, done = run_cpu_pool(work, range(nk), budget_s=10.0)
            res["cpu_baseline"] = {
                "value": evals / dt, "unit": "evals/s", "cores": CPU_THREADS, "kind": "port", "host": host_cpu(),
                "sample": f"{done} keys x 64 points: the reference's Evaluate (one EvaluateAt "
                          f"per level, h:83-105) on the oracle (keygen included), {dt:.1f} s "
                          f"wall on {CPU_THREADS} host threads"}
        print(json.dumps(res), flush=True)
    if group_up(dist):
        dist.destroy_process_group()


def cpu_baseline_heavy_hitters(logs, record, alphas, seeds, top_k, budget_s=15.0):
    """The oracle's EvaluateUntil (C restatement of distributed_point_function.h:
    641-837 + cc:351-498 over OpenSSL AES-NI, one host thread) on a bounded
    sample of the workload: server 0's keys of the first clients, every level,
    at the candidate prefixes the GPU run selected."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from distributed_point_functions_amd import heavy_hitters as HH
    vt = ("tuple", [("intmodn", 32, HH.MODULUS)] * 2)
    P = O.OracleParams([(log, vt, HH.SECURITY_PARAMETER) for log in logs])
    plan, prev = [], []
    for h, vals, counts, _ in record:
        plan.append(prev)
        prev = HH.select(vals, counts, top_k)
    betas = [list(HH.BETA)] * len(logs)

    def keygen(c):
        a = int(alphas[c, 0]) | int(alphas[c, 1]) << 64
        return O.generate_keys(P, a, betas, int(seeds[2 * c, 0]) | int(seeds[2 * c, 1]) << 64,
                               int(seeds[2 * c + 1, 0]) | int(seeds[2 * c + 1, 1]) << 64)[0]

    from concurrent.futures import ThreadPoolExecutor
    n_sample = min(len(alphas), 32 * CPU_THREADS)
    with ThreadPoolExecutor(max_workers=CPU_THREADS) as pool:   # untimed
        keys = list(pool.map(keygen, range(n_sample)))

    def work(c):
        ctx = O.create_context(P, keys[c])
        return sum(O.evaluate_until(P, h, pre, ctx).shape[0] for h, pre in enumerate(plan))

    outs, dt, done = run_cpu_pool(work, range(n_sample), budget_s=budget_s)
    return {"value": outs / dt, "unit": "prefix evals/s", "cores": CPU_THREADS, "kind": "port", "host": host_cpu(),
            "sample": f"{done} clients x all {len(logs)} levels of server 0 at the GPU run's "
                      f"candidates (EvaluateUntil per key, oracle over OpenSSL AES-NI); "
                      f"{dt:.1f} s wall on {CPU_THREADS} host threads"}


def _check_shard(dpf, key, out, rank, world, n, alpha, bits=64):
    """EvaluateAt on a handful of points of this shard must equal the device
    output (cheap, outside the timed region)."""
    import torch
    rng = np.random.default_rng(rank)
    local = sorted({0, n - 1, *map(int, rng.integers(0, n, size=6))})
    if alpha // n == rank:
        local.append(alpha % n)
    words = out.view(torch.int64).view(-1, bits // 64)
    pts = [rank * n + i for i in local]
    got_rows = words[torch.tensor(local, device=out.device)].cpu().numpy().view(np.uint64)
    want_rows = dpf.evaluate_at(key, 0, pts, packed=True).view(np.uint64).reshape(got_rows.shape)
    if not np.array_equal(got_rows, want_rows):
        raise SystemExit(f"rank {rank}: device output disagrees with EvaluateAt at {pts}")


if __name__ == "__main__":
    main()
