#!/bin/bash
# r15 lease Y: the synthetic-benchmark and config-1 lines again on the
# current tree (host-side changes since part 4), as round_evidence's part 4 writes them.
set -u
O=gpurun_out; mkdir -p $O
TAG=r15
line() {
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_${TAG}_$name.log 2>&1 || { tail $O/bench_${TAG}_$name.log; exit 1; }
  grep '^{' $O/bench_${TAG}_$name.log > $O/bench_${TAG}_$name.json
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], d['value'], d['unit'])" $O/bench_${TAG}_$name.json $name
}
line config1 --log-domain 20 --steps 500 --warmup 50
line syn_dev32 --workload synthetic_hierarchical_device --domain 32
line syn_dev128 --workload synthetic_hierarchical_device --domain 128
line syn_h32 --workload synthetic_hierarchical --domain 32
line syn_h128 --workload synthetic_hierarchical --domain 128
line syn_d32 --workload synthetic_direct --domain 32
line syn_d128 --workload synthetic_direct --domain 128
