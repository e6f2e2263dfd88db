#!/bin/bash
# r15 lease Z: config 1's line with enough warmup to bring the GPU to full
# clock (a 50 us step x 50 warmup steps left it at a lower power state when
# the line ran first on a fresh box), twice.
set -u
O=gpurun_out; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --log-domain 20 --steps 2000 --warmup 5000 > $O/bench_r15_config1_r$r.log 2>&1 || exit 1
  grep '^{' $O/bench_r15_config1_r$r.log > $O/bench_r15_config1_r$r.json
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read()); print(d['ms_per_step']*1e3, 'us/step', d['roofline']['launch_ms']*1e3, 'us launch')" $O/bench_r15_config1_r$r.json
done
