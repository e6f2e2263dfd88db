#!/bin/bash
# r14 probe 2: where a slow (~2.7 s) EvaluateUntil<uint128> 2^31 host-output
# call spends its time (DPF_HIP_D2H_TRACE=1: value-initialisation on the
# calling thread, DMA issue, final wait), twelve calls.
set -u
O=gpurun_out; mkdir -p $O
export DPF_HIP_D2H_TRACE=1
for r in 1 2; do
  timeout -k 10 400 python bench.py --workload full_domain_u128 --host-output --host-output-reps 6 --no-cpu-baseline --steps 2 --warmup 1 > $O/reps2_$r.json 2> $O/reps2_$r.err || { tail -5 $O/reps2_$r.err; exit 1; }
  grep pipelined_d2h $O/reps2_$r.err || true
done
