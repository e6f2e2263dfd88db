#!/bin/bash
# One parameterised A/B harness for GPU leases (replaces the per-experiment
# r13_*.sh scripts).  Runs the named pytest files first (parity of what is
# being compared), then `bench.py <args>` once per variant and round, variants
# alternating so box drift hits all of them alike, and prints one line per run:
#   <variant> value unit launch_ms roofline.frac [seconds_per_pass] [api_ms per call]
# A variant is
#   lib:<name>        vlib/<name>.so copied over the in-tree libdpf_hip.so
#                     (built by tools/build_variant.sh), restored afterwards;
#   env:<VAR>=<val>[,<VAR>=<val>...]   the current library with those
#                     environment variables set;
#   cur               the current library, no extra environment.
# Usage (GPU box, repo root):
#   bash tools/ab.sh [--tests "tests/a.py tests/b.py"] [--rounds N] [--tag t] \
#       -- "<bench.py args>" variant1 variant2 ...
set -u
TESTS=""; ROUNDS=2; TAG=ab
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case $1 in
    --tests) TESTS=$2; shift 2 ;;
    --rounds) ROUNDS=$2; shift 2 ;;
    --tag) TAG=$2; shift 2 ;;
    *) echo "ab.sh: unknown option $1"; exit 2 ;;
  esac
done
shift   # --
ARGS=$1; shift
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L $O/.ab_orig.so
restore() { cp $O/.ab_orig.so $L; }
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread \
    > $O/${TAG}_tests.log 2>&1 || { tail -30 $O/${TAG}_tests.log; exit 1; }
  tail -1 $O/${TAG}_tests.log
fi
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    envset=""
    case $v in
      lib:*) cp vlib/${v#lib:}.so $L ;;
      env:*) envset=${v#env:}; envset=${envset//,/ } ;;
      cur) ;;
      *) echo "ab.sh: bad variant $v"; restore; exit 2 ;;
    esac
    log=$O/${TAG}_$(echo $v | tr ':=/,' '____')_r$r.log
    env $envset timeout -k 10 600 python bench.py $ARGS --no-cpu-baseline > $log 2>&1
    rc=$?; restore
    [ $rc -eq 0 ] || { echo "$v failed"; tail -5 $log; exit 1; }
    python3 - "$v" "$log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
r = d.get("roofline", {})
api = d.get("api_level", {})
print(sys.argv[1], f"{d['value']:.4g}", d["unit"], r.get("launch_ms") or r.get("launch_ms_per_pass"),
      f"{r.get('frac', 0):.4f}", d.get("seconds_per_pass", ""),
      f"api_ms {api['api_ms_per_call']}" if api else "")
PY
  done
done
