#!/bin/bash
# r15 lease L: Mod32Leaf<5> parity + the reference grid rows it changes, then evidence part 2.
set -u
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/r15l_tests.log 2>&1
rc=$?; tail -2 $O/r15l_tests.log; [ $rc -eq 0 ] || { tail -30 $O/r15l_tests.log; exit 1; }
timeout -k 10 300 distributed_point_functions_amd/lib/dpf_benchmark '--benchmark_filter=EvaluateRegularDpf<Tuple<MyIntModN x5>>' > $O/r15l_modn5.txt 2>&1 || exit 1
grep BM_ $O/r15l_modn5.txt
bash tools/round_evidence.sh r15 part2
