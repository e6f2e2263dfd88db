#!/bin/bash
# Same-box A/B of two builds of libdpf_hip.so on bench.py workloads that go
# through the host C++ library (which loads the in-tree libdpf_hip.so):
# alternates copying each build in place.  Usage: tools/lib_ab_bench.sh <libA> <libB> <bench args...>
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
A=$1; B=$2; shift 2
T=$R/distributed_point_functions_amd/lib/libdpf_hip.so
cp $T /tmp/orig_libdpf_hip.so
for round in 1 2; do
  for lib in $A $B; do
    cp $R/$lib $T
    echo "== $lib"
    timeout -k 10 300 python $R/bench.py --no-cpu-baseline "$@" 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print(json.dumps({k: d.get(k) for k in ('value','unit','ms_per_step','aes_blocks_per_s')}))" || { cp /tmp/orig_libdpf_hip.so $T; exit 1; }
  done
done
cp /tmp/orig_libdpf_hip.so $T
