#!/bin/bash
# r15 lease AC: phase split of the prefix walk (lookup / upload / device / context)
# in the synthetic hierarchical benchmark (2^20 prefixes per level).
set -u
O=gpurun_out; mkdir -p $O
DPF_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain 32 > $O/r15ac_syn32.json 2> $O/r15ac_syn32.err || exit 1
grep -h "host timing" $O/r15ac_syn32.err
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['unit'])" $O/r15ac_syn32.json
