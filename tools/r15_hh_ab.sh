#!/bin/bash
# r15 lease B: heavy hitters' expansion-cache modes, same box.  2^18 clients
# (a spare fits): spare (default) / permuted in place / gather + in place;
# 2^20 clients (no spare fits): permuted in place (default) / gather.  Then
# the EvaluateAt host-path phases per reference-benchmark case.
set -u
O=gpurun_out; mkdir -p $O
for c in 1/400000 10/40000 100/4000; do
  DPF_HOST_TIMING=1 timeout -k 10 120 distributed_point_functions_amd/lib/dpf_benchmark \
    --benchmark_filter="BatchEvaluation.*/$c\$" > $O/r15b_be_${c/\//_}.txt 2>&1 || exit 1
  cat $O/r15b_be_${c/\//_}.txt
done
bash tools/ab.sh --tag r15b_hh18 --rounds 2 -- "--workload heavy_hitters --keys-log 18" \
  cur env:DPF_BATCH_CACHE_MODE=permute env:DPF_BATCH_CACHE_MODE=gather || exit 1
bash tools/ab.sh --tag r15b_hh20 --rounds 1 -- "--workload heavy_hitters" \
  cur env:DPF_BATCH_CACHE_MODE=gather || exit 1
