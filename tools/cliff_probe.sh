#!/bin/bash
# Where the drop-in API's mid-size time goes (VERDICT r3 "mid-size cliff"):
# the host's CPU limits, THP and malloc settings, then the reference suite's
# failing BM_EvaluateRegularDpf rows with --split (context copy / packed
# evaluation / unpack / free) at several host-thread caps, with the cgroup's
# throttling counters around each run, and one kernel trace.
# Usage (GPU box, repo root): bash tools/cliff_probe.sh <tag>
set -u
TAG=${1:-cliff}
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
B=distributed_point_functions_amd/lib/dpf_benchmark
{
  echo "nproc=$(nproc) affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))') OMP=${OMP_NUM_THREADS:-}"
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.weight /sys/fs/cgroup/cpuset.cpus.effective \
           /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag; do
    echo "$f: $(cat $f 2>/dev/null)"; done
  ldd --version | head -1
} > $O/host.txt 2>&1
cat $O/host.txt
F='^BM_EvaluateRegularDpf<(uint64_t>/(20|22|24)|uint128>/(20|22)|Tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t>>/(18|20|22)|Tuple<uint64_t, uint64_t>>/(18|20|22)|XorWrapper<uint128>>/(20|22))$'
for th in 16 4 1; do
  echo "== DPF_HOST_THREADS=$th" >> $O/split.txt
  grep -E 'nr_throttled|throttled_usec' /sys/fs/cgroup/cpu.stat >> $O/split.txt 2>/dev/null
  DPF_HOST_THREADS=$th timeout -k 10 240 $B --split "--benchmark_filter=$F" >> $O/split.txt 2>&1 || { echo "split th=$th failed"; exit 1; }
  grep -E 'nr_throttled|throttled_usec' /sys/fs/cgroup/cpu.stat >> $O/split.txt 2>/dev/null
done
cat $O/split.txt
DPF_HOST_TIMING=1 timeout -k 10 240 $B "--benchmark_filter=$F" > $O/bench.txt 2>&1 || { echo "bench failed"; tail $O/bench.txt; exit 1; }
cat $O/bench.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o cliff --output-format csv -- $B --split "--benchmark_filter=$F" > $O/trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo done
