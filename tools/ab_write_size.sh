#!/bin/bash
# Same-box A/B of kernel libraries vlib/<name>.so on the config-2 bench: step
# time (two alternating rounds) and WRITE_SIZE per octet-kernel launch
# (rocprofv3 --pmc, 6 launches).  Usage: tools/ab_write_size.sh name1 name2 ...
set -u
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
L=distributed_point_functions_amd/lib/libdpf_hip.so
cp $L vlib/_orig.so
for r in 1 2; do
  bash tools/ab_lib.sh "--steps 10 --warmup 2" "$@" || exit 1
done
for v in "$@"; do
  cp vlib/$v.so $L
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/wa_$v -o wa --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/wa_$v.log 2>&1 || { cp vlib/_orig.so $L; echo "pmc $v failed"; exit 1; }
  python3 - <<PY
import csv, glob
rows=[r for f in glob.glob("$O/wa_$v/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f)) if "expand_octet" in r["Kernel_Name"]]
ws=[float(r["Counter_Value"]) for r in rows if r["Counter_Name"]=="WRITE_SIZE"]
print("$v", "launches", len(ws), "WRITE_SIZE GB/launch", sum(ws)/max(len(ws),1)*1024/1e9)
PY
done
cp vlib/_orig.so $L
