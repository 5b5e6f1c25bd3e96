"""Bytes per launch of the bench's probed kernels from the rocprofv3 --pmc passes of tools/pmc_traffic.sh.
bytes = (2 * FETCH_SIZE + WRITE_SIZE) KB * 1024: FETCH_SIZE counts half the bytes of wide coalesced reads on
gfx950 (MI355X_MICROARCH.md, HBM section); L2 memory-side traffic, Infinity-Cache hits included.
python tools/pmc_summary.py <dir with {tgn,tgnn}_{fetch,write}/run_counter_collection.csv>"""
import csv
import glob
import json
import os
import sys

# probe name (bench.py kernels_us) -> substrings that select its rocprof kernel name
KERNELS = {
    "tgn_gru_edge": ("gemmN_kernel", "LoadGruA,"),
    "tgn_wgrad_dz0": ("gemmN_kernel", "LoadZ1T", "EpiGruBwd"),
    "tgn_attn_fwd": ("tgn_attn_fwd<true>",),
    "tgn_attn_bwd": ("tgn_attn_bwd",),
    "tgn_kv_dE": ("gemmN_kernel", "KvReduceJob"),
    "tgn_proj": ("gemmN_kernel", "LoadProjW,"),
    "tgn_wgrad3": ("gemmN_kernel", "SnapJob"),
    "tgn_agg_emit": ("tgn_agg_emit",),
    "tgn_scan": ("tgn_scan<true>",),
    "tgn_mark": ("tgn_mark<true>",),
    "tgn_pred_train": ("tgn_pred_train",),
    "tgn_fixup_update": ("gemm_fixup_kernel<tgnx::tgn::TrainTail",),
    "tgn_adam": ("tgn_adam",),
    "tgnn_edge_fwd": ("tgnn_edge_fwd",),
    "tgnn_edge_bwd": ("tgnn_edge_bwd",),
    "tgnn_seg_fwd": ("tgnn_seg_fwd<true>",),
    "tgnn_seg_bwd": ("tgnn_seg_bwd_pred",),
    "tgnn_pred_train": ("tgnn::tgnn_pred_train", "tgnx::tgnn_pred_train"),
    "tgnn_assemble": ("tgnn_assemble<true>",),
}


def load(path, counter=None, win=None):
    """kernel name -> list of per-dispatch counter values (KB; raw counters: counts), one counter per call, in
    dispatch order; win = "a:b": only dispatches [a, b) of each kernel (a kernel launched once per step: the bench
    line's config.timed_steps, i.e. the timed window's steps; PMC_WINDOW_TGN / PMC_WINDOW_TGNN)"""
    out = {}
    rows = list(csv.DictReader(open(path)))
    if rows and "Dispatch_Id" in rows[0]:
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        if counter is None or r["Counter_Name"] == counter:
            out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    if win:
        a, b = (int(x) for x in win.split(":"))
        out = {k: v[a:b] for k, v in out.items() if v[a:b]}
    return out


# exact memory-side bytes from the raw request counters (tools/pmc_calib.hip on the box: every coalesced read
# width — 4, 8, 16 B per lane — goes out as 128-B requests, counted in TCC_EA0_RDREQ_128B; FETCH_SIZE tallies
# them at 64 B, hence its factor 2; writes are 64-B or 32-B requests and WRITE_SIZE is exact):
#   read  = 128 RDREQ_128B + 64 RDREQ_64B + 32 RDREQ_32B      (RDREQ = their sum)
#   write = 64 WRREQ_64B + 32 (WRREQ - WRREQ_64B)
RAW_RD = {"TCC_EA0_RDREQ_128B_sum": 128, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_32B_sum": 32}


def raw_bytes(rd_csv, wr_csv, keys, win=None):
    """per-launch (read, write, 64-B read requests) bytes of the kernels matching keys, or None"""
    rd = 0.0
    n64 = 0.0
    for ctr, sz in RAW_RD.items():
        t = load(rd_csv, ctr, win)
        v = [x for n in t if match(n, keys) for x in t[n]]
        if not v:
            return None
        rd += sz * sum(v) / len(v)
        if sz == 64:
            n64 = sum(v) / len(v)
    tw, t64 = load(wr_csv, "TCC_EA0_WRREQ_sum", win), load(wr_csv, "TCC_EA0_WRREQ_64B_sum", win)
    w = [x for n in tw if match(n, keys) for x in tw[n]]
    w64 = [x for n in t64 if match(n, keys) for x in t64[n]]
    if not w or not w64:
        return None
    a, b = sum(w) / len(w), sum(w64) / len(w64)
    return rd, 64 * b + 32 * (a - b), n64


def match(name, keys):
    if keys[0] == "tgnn::tgnn_pred_train":  # either spelling
        return any(k in name for k in keys)
    return all(k in name for k in keys)


def main(d):
    res = {"_note": __doc__.split("\n")[1] + " " + __doc__.split("\n")[2]}
    for model in ("tgn", "tgnn"):
        f = glob.glob(os.path.join(d, f"{model}_fetch", "**", "*counter_collection.csv"), recursive=True)
        w = glob.glob(os.path.join(d, f"{model}_write", "**", "*counter_collection.csv"), recursive=True)
        win = os.environ.get(f"PMC_WINDOW_{model.upper()}")
        if win:
            res[f"_window_{model}"] = f"dispatches [{win.replace(':', ', ')}) of each kernel: the timed steps"
        fe, wr = (load(f[0], win=win), load(w[0], win=win)) if f and w else ({}, {})
        for probe, sel in KERNELS.items():
            if not fe or not probe.startswith(model + "_"):
                continue
            fkb = wkb = 0.0
            launches = None
            for keys in (sel if isinstance(sel, list) else [sel]):   # several kernels: per-launch sums
                fn = [n for n in fe if match(n, keys)]
                wn = [n for n in wr if match(n, keys)]
                if not fn or not wn:
                    break
                fv = [v for n in fn for v in fe[n]]
                wv = [v for n in wn for v in wr[n]]
                fkb += sum(fv) / len(fv)
                wkb += sum(wv) / len(wv)
                launches = len(fv) if launches is None else min(launches, len(fv))
            else:
                res[probe] = {"fetch_kb": round(fkb, 2), "write_kb": round(wkb, 2), "launches": launches,
                              "bytes_per_launch": int((2 * fkb + wkb) * 1024)}
        rf = glob.glob(os.path.join(d, f"{model}_rd", "**", "*counter_collection.csv"), recursive=True)
        rw = glob.glob(os.path.join(d, f"{model}_wr", "**", "*counter_collection.csv"), recursive=True)
        if rf and rw:
            for probe, sel in KERNELS.items():
                if not probe.startswith(model + "_"):
                    continue
                r = raw_bytes(rf[0], rw[0], sel, win)
                if r is None:
                    continue
                e = res.setdefault(probe, {})
                e["raw_read_bytes"], e["raw_write_bytes"], e["raw_rdreq_64b"] = int(r[0]), int(r[1]), int(r[2])
                e["raw_bytes_per_launch"] = int(r[0] + r[1])
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
