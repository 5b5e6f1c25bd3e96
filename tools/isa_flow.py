"""Per-basic-block sequence of memory / wait / barrier / MFMA ops of one kernel in a hipcc -save-temps
device .s:  python tools/isa_flow.py file.s <symbol-prefix>"""
import re
import sys

lines = open(sys.argv[1]).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(sys.argv[2]) and ":" in l and not l.startswith("\t"))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
bb, cnt, order = "entry", {"entry": []}, ["entry"]
KEEP = ("global_load", "global_store", "buffer_load", "s_waitcnt", "s_barrier", "v_mfma", "ds_", "s_cbranch",
        "s_branch", "global_atomic")
for l in lines[start + 1:end]:
    m = re.match(r"^(\.LBB\S+):", l)
    if m:
        bb = m.group(1)
        order.append(bb)
        cnt[bb] = []
        continue
    s = l.strip().replace("\t", " ")
    if s.startswith(KEEP):
        cnt[bb].append(s)
for b in order:
    out, prev, n = [], None, 0
    for s in cnt[b]:
        k = s if s.startswith(("s_waitcnt", "s_cbranch", "s_branch")) else s.split()[0]
        if k == prev:
            n += 1
        else:
            if prev:
                out.append(f"{prev} x{n}" if n > 1 else prev)
            prev, n = k, 1
    if prev:
        out.append(f"{prev} x{n}" if n > 1 else prev)
    if out:
        print(b, " | ".join(out))
