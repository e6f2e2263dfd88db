#!/bin/bash
# Octet expand kernel at forced subtree depths S (DFS stack = S - 3 levels in
# scratch): config-2 step time (bench.py, two alternating rounds) and the
# WRITE_SIZE of each (rocprofv3 --pmc, 5 timed launches), i.e. whether a
# shallower DFS stack keeps its pushes in L2.
set -u
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
for r in 1 2; do
  bash tools/ab_lib.sh "--steps 10 --warmup 2" s9 s10 s11 s12 || exit 1
done
for v in s9 s10 s11 s12; do
  cp vlib/$v.so $L
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/wa_$v -o wa --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/wa_$v.log 2>&1 || { cp vlib/_orig.so $L; echo "pmc $v failed"; exit 1; }
  python3 - <<PY
import csv, glob
rows=[r for f in glob.glob("$O/wa_$v/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f)) if "expand_octet" in r["Kernel_Name"]]
ws=[float(r["Counter_Value"]) for r in rows if r["Counter_Name"]=="WRITE_SIZE"]
print("$v", "launches", len(ws), "WRITE_SIZE KiB/launch", sum(ws)/max(len(ws),1), "-> GB", sum(ws)/max(len(ws),1)*1024/1e9)
PY
done
cp vlib/_orig.so $L
