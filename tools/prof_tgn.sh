#!/bin/bash
# On the GPU box: rocprofv3 kernel stats of the TGN wiki bench (graph replay) -> gpurun_out/<tag>_prof/, and a
# per-step kernel table (kernels launched once per step) on stdout.
tag=${1:-pt}
R=/root/repo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${tag}_prof -o run -- \
  python3 $R/bench.py --model tgn --only --steps 200 --warmup 20 --no-cpu-baseline ${EXTRA} \
  > $R/gpurun_out/${tag}_prof.json 2> $R/gpurun_out/${tag}_prof.err || exit $?
python3 - $R/gpurun_out/${tag}_prof <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
steps = max(int(r["Calls"]) for r in rows if "tgn_pred_train" in r["Name"])
tot = 0
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    c = int(r["Calls"]); a = float(r["AverageNs"]) / 1e3
    if c >= steps * 0.9:
        tot += a * c / steps
        print(f"{r['Name'][:110]:110s} {c:6d} {a:8.2f}us")
print("steps %d, per-step kernel sum %.1f us" % (steps, tot))
PY
