#!/bin/bash
# A/B of host-library variants on one GPU box: vlib/host_<name>/ holds a
# libdpf.so and _dpf_host*.so built from one tree; each variant is copied
# over the in-tree ones for its runs (alternating, so box drift hits all
# alike), the in-tree pair restored afterwards.  One line per run:
#   <variant> <bench.py args> value unit
# Usage (GPU box, repo root):
#   bash tools/host_ab.sh [--tests "tests/a.py"] [--rounds N] -- "<bench.py args>" [...] -- name1 name2 ...
set -u
TESTS=""; ROUNDS=2
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in
    --tests) TESTS=$2; shift 2 ;;
    --rounds) ROUNDS=$2; shift 2 ;;
    *) echo "host_ab.sh: unknown option $1"; exit 2 ;;
  esac
done
shift
ARGSETS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARGSETS+=("$1"); shift; done
shift
O=gpurun_out; mkdir -p $O/host_ab_orig
L=distributed_point_functions_amd/lib
cp $L/libdpf.so $L/_dpf_host*.so $O/host_ab_orig/
restore() { cp $O/host_ab_orig/* $L/; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
    > $O/host_ab_tests.log 2>&1 || { tail -30 $O/host_ab_tests.log; exit 1; }
  tail -1 $O/host_ab_tests.log
fi
for r in $(seq 1 $ROUNDS); do
  for a in "${ARGSETS[@]}"; do
    for v in "$@"; do
      cp vlib/host_$v/* $L/
      log=$O/host_ab_${v}_r$r.log
      timeout -k 10 600 python bench.py $a --no-cpu-baseline > $log 2>&1
      rc=$?; restore
      [ $rc -eq 0 ] || { echo "$v failed"; tail -5 $log; exit 1; }
      python3 -c "
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][-1])
print(sys.argv[1], sys.argv[3], f\"{d['value']:.4g}\", d['unit'])" "$v" "$log" "$a"
    done
  done
done
