set -o pipefail
mkdir -p gpurun_out/ws1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "ws" -x -v --timeout 120 --timeout-method thread > gpurun_out/ws1/tests.log 2>&1; rc=$?
tail -5 gpurun_out/ws1/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ws1/bench.json 2>gpurun_out/ws1/bench.err; rc=$?
cat gpurun_out/ws1/bench.json; exit $rc
