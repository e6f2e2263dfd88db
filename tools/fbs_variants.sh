#!/bin/bash
# Builds the fbs_microbench variants: mode ff_lds ff_glb sbox_group waves no_ff
cd "$(dirname "$0")"
build() {
  local name=fbsm_$1_$2_$3_$4_$5_$6
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DFBS_MODE=$1 -DFBS_FF_LDS=$2 -DFBS_FF_GLB=$3 \
    -DFBS_SBOX_GROUP=$4 -DFBS_WAVES=$5 -DFBS_NO_FF=$6 fbs_microbench.hip -o $name \
    -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "error|VGPRs: |VGPRs Spill|Occupancy" \
    | sed 's/.*remark: *//;s/ \[-Rpass.*\]//' | tr '\n' ' ' | sed "s/^/$name: /"; echo
}
for v in "$@"; do build $v; done
