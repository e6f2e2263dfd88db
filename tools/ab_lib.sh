#!/bin/bash
# A/B of kernel libraries on one box: each vlib/<name>.so is copied over the
# in-tree libdpf_hip.so in turn and `bench.py <args>` is run; prints value and
# launch_ms per run.  Usage: tools/ab_lib.sh "<bench args>" name1 name2 ...
set -u
ARGS=$1; shift
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
for v in "$@"; do
  cp vlib/$v.so $L
  timeout -k 10 400 python bench.py $ARGS --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || { cp vlib/_orig.so $L; exit 1; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_$v.log') if l.startswith('{')][0]); print('$v', d['value'], d['unit'], d.get('roofline',{}).get('launch_ms'))"
done
cp vlib/_orig.so $L
