#!/bin/bash
# r14 probe: per-call time of EvaluateUntil<T> -> fresh host vector, T =
# uint128 (2^31 outputs, 32 GiB) and uint64 (2^30, 8 GiB), six calls each,
# under the pipelined copy (default pieces), 256 MiB pieces, and the
# whole-range registration (DPF_HIP_D2H_PIPELINE=0); DPF_HIP_D2H_TRACE=1 splits
# each pipelined call into mapping, registering and waiting.
set -u
O=gpurun_out; mkdir -p $O
T=tests/test_api_gpu.py
timeout -k 10 600 python -u -m pytest $T::test_pipelined_host_output_and_its_fallbacks $T::test_split_first_call_then_next_level $T::test_concurrent_pipelined_host_outputs $T::test_large_host_output_matches_device tests/test_host_copies_gpu.py -x -q --timeout 300 --timeout-method thread > $O/reps_tests.log 2>&1 || { tail -30 $O/reps_tests.log; exit 1; }
tail -1 $O/reps_tests.log
export DPF_HIP_D2H_TRACE=1
for w in full_domain_u128 full_domain; do
for v in "cur:DPF_NOTHING=0" "piece256:DPF_HIP_D2H_PIECE_MIB=256" "pipe0:DPF_HIP_D2H_PIPELINE=0" "cur2:DPF_NOTHING=0"; do
  name=${w}_${v%%:*}; E=${v#*:}
  env $E timeout -k 10 400 python bench.py --workload $w --host-output --host-output-reps 6 --no-cpu-baseline --steps 2 --warmup 1 > $O/reps_$name.json 2> $O/reps_$name.err || { tail -5 $O/reps_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], [round(x) for x in d['api_level']['api_ms_per_call']])" $O/reps_$name.json $name
  grep pipelined_d2h $O/reps_$name.err | tail -1 || true
done
done
