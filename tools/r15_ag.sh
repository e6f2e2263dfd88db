#!/bin/bash
# r15 lease AG: the whole -m gpu suite and smoke() on the committed final tree.
set -u
O=gpurun_out; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/r15ag_gpu_tests.log 2>&1 || { tail -30 $O/r15ag_gpu_tests.log; exit 1; }
tail -1 $O/r15ag_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r15ag_smoke.log 2>&1 || { cat $O/r15ag_smoke.log; exit 1; }
cat $O/r15ag_smoke.log
