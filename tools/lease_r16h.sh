export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_batch_context_gpu.py tests/test_heavy_hitters_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r16j_tests.log 2>&1; rc=$?; tail -2 $O/r16j_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab.sh --tag r16j_hh20 --rounds 2 -- "--workload heavy_hitters" cur lib:hhnt || exit 1
