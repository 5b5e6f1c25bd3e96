"""Mean counter value per dispatch, by kernel (short name), from rocprofv3 --pmc csv directories.
    python tools/pmc_kernels.py <dir> [<dir> ...]"""
import csv
import glob
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(tgn_\w+|gemmN_kernel|gemm_fixup_kernel|tgnn_\w+|gemm\w*)", name)
    return m.group(1) if m else name[:40]


tot = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(set))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r.get("Kernel_Name", ""))
            c = r.get("Counter_Name")
            tot[k][c] += float(r.get("Counter_Value", 0))
            cnt[k][c].add(r.get("Dispatch_Id"))
for k in sorted(tot):
    vals = {c: tot[k][c] / max(len(cnt[k][c]), 1) for c in tot[k]}
    print(k, " ".join(f"{c}={v:.4g}" for c, v in sorted(vals.items())))
