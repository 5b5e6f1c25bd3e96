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


def load(path):
    """kernel name -> list of per-dispatch counter values (KB)"""
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return out


def match(name, keys):
    if keys[0] == "tgnn::tgnn_pred_train":  # either spelling
        return any(k in name for k in keys)
    return all(k in name for k in keys)


def main(d):
    res = {"_note": __doc__.split("\n")[1] + " " + __doc__.split("\n")[2]}
    for model in ("tgn", "tgnn"):
        f = glob.glob(os.path.join(d, f"{model}_fetch", "**", "*counter_collection.csv"), recursive=True)
        w = glob.glob(os.path.join(d, f"{model}_write", "**", "*counter_collection.csv"), recursive=True)
        if not f or not w:
            continue
        fe, wr = load(f[0]), load(w[0])
        for probe, sel in KERNELS.items():
            if not probe.startswith(model + "_"):
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
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
