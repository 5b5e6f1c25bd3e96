"""Per-kernel median / p10 / p90 durations (us) from a rocprofv3 kernel_trace.csv."""
import csv
import sys
from collections import defaultdict

import numpy as np

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(d.items(), key=lambda kv: -np.median(kv[1]) * len(kv[1]))
for name, v in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    v = np.array(v)
    print(f"{name[:90]:90s} n={len(v):5d} med={np.median(v):7.2f} p10={np.percentile(v, 10):7.2f} p90={np.percentile(v, 90):7.2f}")
