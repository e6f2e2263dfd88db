#!/bin/bash
# WRITE_SIZE / FETCH_SIZE of the config-2 expand kernel for each library given
# (tools/expand_ab.py --one); per-dispatch counters in gpurun_out/wpmc/<name>/.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  n=$(basename $lib .so)
  O=$R/gpurun_out/wpmc/$n; mkdir -p $O
  DPF_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $O/w -o w --output-format csv -- python3 $R/tools/expand_ab.py --one --reps 2 ${WPMC_ARGS:-} > $O/w.log 2>&1 || exit 1
  DPF_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format csv -- python3 $R/tools/expand_ab.py --one --reps 2 ${WPMC_ARGS:-} > $O/f.log 2>&1 || exit 1
done
echo ok
