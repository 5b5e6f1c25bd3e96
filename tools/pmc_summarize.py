"""Average FETCH_SIZE / WRITE_SIZE per launch for the kernels bench.py prices (profiles/pmc_traffic.json).

traffic bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B): the gfx950 correction of MI355X_MICROARCH.md
(HBM section: FETCH_SIZE counts half the bytes of wide coalesced reads; WRITE_SIZE is exact for
streaming stores and float atomics).  Other access widths are uncalibrated there; the json says so.
Infinity-Cache hits are counted by these fabric-side counters (same section)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# bench.py probe name -> substrings that identify the launch's kernel in the rocprof name
KEYS = {
    "tgn_gru_edge": ["LoadGruA", "LoadEdgeAttr"],
    "tgn_attn_fwd": ["tgn_attn_fwd"],
    "tgn_attn_bwd": ["tgn_attn_bwd"],
    "tgn_agg_emit": ["tgn_agg_emit"],
    "tgn_wgrad_dz0": ["gemmN_kernel", "LoadEdgeAttrT", "LoadProjWT"],
    "tgnn_edge_fwd": ["tgnn_edge_fwd"],
    "tgnn_edge_bwd": ["tgnn_edge_bwd"],
    "tgnn_seg_fwd": ["tgnn_seg_fwd"],
    "tgnn_seg_bwd_pred": ["tgnn_seg_bwd_pred"],
}


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r.get("Counter_Name") != counter:
            continue
        per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return per


def match(per, subs):
    vals = []
    for name, v in per.items():
        if all(s in name for s in subs):
            vals += v
    return vals


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
out = {"_note": "bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KB * 1024, averaged over launches; FETCH x2 is the "
                "gfx950 correction for wide coalesced reads (MI355X_MICROARCH.md HBM section), other widths "
                "uncalibrated; L2-miss (fabric-side) traffic, Infinity-Cache hits included"}
for probe, subs in KEYS.items():
    fv, wv = match(fetch, subs), match(write, subs)
    if not fv or not wv:
        continue
    f_kb, w_kb = sum(fv) / len(fv), sum(wv) / len(wv)
    out[probe] = {"fetch_kb": round(f_kb, 2), "write_kb": round(w_kb, 2), "launches": len(fv),
                  "bytes_per_launch": round((2 * f_kb + w_kb) * 1024)}
prev = json.load(open(sys.argv[3])) if os.path.exists(sys.argv[3]) else {}
prev.update(out)                                   # one file for both paths' probes
json.dump(prev, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
