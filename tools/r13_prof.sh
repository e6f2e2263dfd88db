#!/bin/bash
# rocprofv3 kernel trace + PMC passes of the DCF bench (r13dcf) and of one
# 2^18-client heavy-hitters pass (r13hh) on the current tree.
set -u
export TMPDIR=/tmp
bash profiles/profile.sh r13dcf --workload dcf --steps 5 --warmup 1 --no-cpu-baseline || exit 1
bash profiles/profile.sh r13hh --workload heavy_hitters --keys-log 18 --steps 1 --warmup 0 --no-cpu-baseline || exit 1
echo all ok
