#!/bin/bash
# Every bench.py workload once on one GPU (outputs under gpurun_out/bench_<tag>_*.json).
set -u
TAG=${1:-r06}
O=gpurun_out
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > $O/bench_${TAG}_$name.log 2>&1; local rc=$?; grep '^{' $O/bench_${TAG}_$name.log > $O/bench_${TAG}_$name.json; echo "$name rc=$rc"; return $rc; }
run full_domain && run full_domain_u128 --workload full_domain_u128 && \
run tuple_mod --workload full_domain_tuple --tuple-type intmodn32x2 && run tuple_u32 --workload full_domain_tuple --tuple-type u32x2 && \
run evaluate_at --workload evaluate_at && \
run evaluate_at_sum --workload evaluate_at_sum && run dcf --workload dcf && \
run heavy_hitters --workload heavy_hitters && \
run syn_dev32 --workload synthetic_hierarchical_device --domain 32 && run syn_dev128 --workload synthetic_hierarchical_device --domain 128 && \
run syn_h32 --workload synthetic_hierarchical --domain 32 && run syn_h128 --workload synthetic_hierarchical --domain 128 && \
run syn_d32 --workload synthetic_direct --domain 32 && run syn_d128 --workload synthetic_direct --domain 128
