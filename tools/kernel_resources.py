#!/usr/bin/env python3
"""Compact per-kernel resource table (VGPRs, AGPRs, scratch, occupancy) of
dpf_kernels.hip from hipcc's -Rpass-analysis=kernel-resource-usage remarks."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "distributed_point_functions_amd", "csrc", "kernels",
                   os.environ.get("KRES_TU", "dpf_kernels.hip"))
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
       f"-I{ROOT}/include", SRC, "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/tmp").stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*)$", line)
    if not m:
        continue
    r = m.group(1).split(" [-Rpass")[0].strip()
    if r.startswith("Function Name:"):
        name = r.split(":", 1)[1].split("[")[0].strip()
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dem = re.sub(r"\(anonymous namespace\)::", "", dem)
        cur = {"name": dem.split("(")[0] if "(" in dem else dem}
        rows.append(cur)
    elif cur is not None:
        for key in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "TotalSGPRs", "VGPRs Spill"):
            if r.startswith(key + ":"):
                cur[key] = r.split(":", 1)[1].strip()
flt = sys.argv[1] if len(sys.argv) > 1 else ""
for c in rows:
    if flt in c["name"]:
        print(f'{c.get("VGPRs","?"):>4} v {c.get("AGPRs","?"):>3} a {c.get("TotalSGPRs","?"):>3} s '
              f'scratch {c.get("ScratchSize [bytes/lane]","?"):>4} occ {c.get("Occupancy [waves/SIMD]","?")}  {c["name"]}')
