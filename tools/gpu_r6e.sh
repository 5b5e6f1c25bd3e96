#!/bin/bash
# per-kernel comparison of the comment-shaped 2-hop step (B = 600) across libraries (rocprofv3 kernel stats)
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r6e}
for lib in default r4 r5; do
  if [ $lib = default ]; then unset TGNX_LIB; else export TGNX_LIB=/root/repo/var/$lib/libtgnx.so; fi
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/${T}_prof_$lib -o run -- \
    python3 /root/repo/bench.py --model tgn --only --no-probe --no-cpu-baseline --no-train-loop --no-tcsr \
    --dataset tgbl-comment --batch 600 --layers 2 --steps 100 --warmup 20 --window start \
    > /root/repo/gpurun_out/${T}_$lib.json 2> /root/repo/gpurun_out/${T}_$lib.err) || exit 1
done
unset TGNX_LIB
python3 - <<'PY'
import csv, glob
rows = {}
for lib in ("default", "r4", "r5"):
    f = glob.glob(f"/root/repo/gpurun_out/r6e_prof_{lib}/**/run_kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if int(r["Calls"]) >= 100:
            rows.setdefault(r["Name"][:120], {})[lib] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
for n, v in sorted(rows.items(), key=lambda kv: -max(x[1] for x in kv[1].values())):
    print(f"{n[:100]:100s}", "  ".join(f"{l}:{v[l][0]}x{v[l][1]:.2f}" if l in v else f"{l}:-" for l in ("default", "r4", "r5")))
PY
