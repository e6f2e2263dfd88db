#!/bin/bash
# Runs every built tools/fbsm_* variant (GPU box); one JSON line each.
# Usage: bash tools/fbs_run.sh <tag> [iters]
TAG=${1:-fbs}; IT=${2:-16}
O=gpurun_out; mkdir -p $O
for b in tools/fbsm_*; do
  [ -x "$b" ] || continue
  echo "# $b" >> $O/${TAG}.txt
  timeout -k 5 60 "$b" $IT >> $O/${TAG}.txt 2>&1 || { echo "FAILED rc=$? $b" >> $O/${TAG}.txt; exit 1; }
done
cat $O/${TAG}.txt
