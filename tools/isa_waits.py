"""Per-kernel load / wait / branch counts from a hipcc -save-temps device .s (serialised loads show as
many `s_waitcnt vmcnt(0)` per global load).  python tools/isa_waits.py file.s [name-filter]"""
import re
import sys

cur, stats = None, {}
for line in open(sys.argv[1]):
    m = re.match(r"^(_Z\S+):", line)
    if m and not line.startswith("\t"):
        cur = m.group(1)
        stats[cur] = [0, 0, 0, 0]
        continue
    if line.startswith(".Lfunc_end"):
        cur = None
    if cur is None:
        continue
    s = stats[cur]
    if "global_load" in line or "buffer_load" in line:
        s[0] += 1
    if "s_waitcnt vmcnt(0)" in line:
        s[1] += 1
    if "s_cbranch" in line:
        s[2] += 1
    if "global_atomic" in line:
        s[3] += 1
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for k, (ld, w, br, at) in stats.items():
    if flt in k:
        print(f"loads {ld:4d} vmcnt0 {w:4d} branches {br:4d} atomics {at:3d}  {k[:110]}")
