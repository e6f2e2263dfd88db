#!/bin/bash
# Builds libdpf_hip.so with extra compiler flags into vlib/<name>.so for
# A/B timing (tools/variant_bench.py, or copied over the in-tree library on a
# scratch GPU box).  Usage: tools/build_variant.sh <name> [flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
out=vlib/$name; mkdir -p $out
K=distributed_point_functions_amd/csrc/kernels
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -mcode-object-version=5 -Iinclude"
for src in $K/*.hip; do
  b=$(basename $src .hip)
  sched="-mllvm -amdgpu-sched-strategy=${DPF_SCHED:-iterative-ilp}"
  # dpf_batch.hip uses the default scheduler unless DPF_BATCH_ILP=1.
  [ "$b" = dpf_batch ] && [ "${DPF_BATCH_ILP:-0}" != 1 ] && sched=""
  /opt/rocm/bin/hipcc $F $sched "$@" -c $src -o $out/$b.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $out/*.o -o vlib/$name.so
rm -rf $out
echo vlib/$name.so
