#!/bin/bash
# Bench lines and rocprofv3 passes for the octet-kernel workloads other than
# the default one (uint128, Tuple<IntModN32 x2>, Tuple<u32,u32>).
# Usage: bash tools/octet_refresh.sh <tag>
set -u
TAG=${1:-r11g}
O=gpurun_out; mkdir -p $O
b() { local name=$1; shift; timeout -k 10 300 python bench.py "$@" > $O/${TAG}_$name.json 2> $O/${TAG}_$name.err || { echo "$name failed"; tail -5 $O/${TAG}_$name.err; exit 1; }; echo "$name ok"; }
b full_domain_u128 --workload full_domain_u128
b tuple_mod --workload full_domain_tuple --tuple-type intmodn32x2
b tuple_u32 --workload full_domain_tuple --tuple-type u32x2
bash profiles/profile.sh ${TAG}tm --workload full_domain_tuple --tuple-type intmodn32x2 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash profiles/profile.sh ${TAG}tu --workload full_domain_tuple --tuple-type u32x2 --steps 5 --warmup 1 --no-cpu-baseline || exit 1
echo all ok
