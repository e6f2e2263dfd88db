export TMPDIR=/tmp; O=gpurun_out; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r16i_gpu_tests.log 2>&1; rc=$?; tail -2 $O/r16i_gpu_tests.log; [ $rc -eq 0 ] || exit 1
for d in 128 32; do
  DPF_BATCH_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical_device --domain $d > $O/r16i_syn_dev$d.json 2> $O/r16i_syn_dev$d.err || exit 1
  DPF_HOST_TIMING=1 timeout -k 10 300 python bench.py --workload synthetic_hierarchical --domain $d > $O/r16i_syn_h$d.json 2> $O/r16i_syn_h$d.err || exit 1
done
bash tools/ab.sh --tag r16i_hh20 --rounds 1 -- "--workload heavy_hitters" cur lib:hhnt || exit 1
