#!/usr/bin/env python3
"""LDS-latency statistics of one kernel in a hipcc -S listing: instructions,
ds_read count, s_waitcnt count, the lgkmcnt(N) histogram (how many LDS reads a
wave keeps in flight between waits), scalar loads, VGPRs and occupancy.

  hipcc --offload-arch=gfx950 -O3 ... --offload-device-only -S x.hip -o x.s
  python tools/isa_stats.py x.s <mangled-name substring>
"""
import collections
import re
import sys


def body(lines, sub):
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sub in l.split(":")[0])
    name = lines[st].split(":")[0]
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".size") and name in lines[i])
    meta = [l for l in lines[en:en + 400] if re.search(r"; (NumVgprs|Occupancy|ScratchSize|NumSgprs):", l)]
    return name, lines[st:en], meta


def main():
    lines = open(sys.argv[1]).read().split("\n")
    name, b, meta = body(lines, sys.argv[2])
    ins = [l for l in b if l.startswith("\t") and not l.startswith("\t.") and not l.strip().startswith(";")]
    txt = "\n".join(ins)
    hist = collections.Counter(int(x) for x in re.findall(r"lgkmcnt\((\d+)\)", txt))
    print(name)
    print(f"instructions {len(ins)}  ds_read {txt.count('ds_read')}  s_waitcnt {txt.count('s_waitcnt')}  "
          f"s_load {txt.count('s_load')}  v_readlane/writelane {len(re.findall('v_(read|write)lane', txt))}  "
          f"scratch {len(re.findall('scratch_', txt))}")
    print("lgkmcnt histogram:", sorted(hist.items()))
    print("\n".join(m.strip() for m in meta))


if __name__ == "__main__":
    main()


def regions(path, sub):
    """Per basic-block-run (between loop labels) ds_read / s_waitcnt counts."""
    lines = open(path).read().split("\n")
    name, b, _ = body(lines, sub)
    cur, rows = None, []
    for l in b:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)$", l)
        if m:
            cur = [m.group(1), m.group(2).strip()[:40], 0, 0, 0, 0]
            rows.append(cur)
        elif cur is not None and l.startswith("\t") and not l.startswith("\t."):
            cur[2] += 1
            cur[3] += "ds_read" in l
            cur[4] += "s_waitcnt" in l and "lgkmcnt" in l
            cur[5] += "v_" in l
    for r in rows:
        if r[3]:
            print(f"{r[0]:>12} ins {r[2]:5d} ds_read {r[3]:4d} lgkm_waits {r[4]:4d} valu {r[5]:5d}  {r[1]}")


if __name__ == "__main__" and len(sys.argv) > 3 and sys.argv[3] == "--regions":
    regions(sys.argv[1], sys.argv[2])
