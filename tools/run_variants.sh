#!/bin/bash
# On the GPU box: bench each build_var/<name>/libtgnx.so (eager, probes on) -> gpurun_out/var_<name>.log
cd "$(dirname "$0")/.."
EXTRA=${EXTRA:-}
for d in build_var/*/; do
  n=$(basename $d)
  TGNX_LIB=$PWD/$d/libtgnx.so timeout -k 10 120 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-graph $EXTRA \
    > gpurun_out/var_$n.log 2>&1 || { echo "variant $n failed rc=$?"; exit 1; }
  python - "$n" <<'PY'
import json, sys
for l in open(f"gpurun_out/var_{sys.argv[1]}.log"):
    if l.startswith("{"):
        j = json.loads(l)
        print(sys.argv[1], j["value"], {k: round(v, 1) for k, v in j["kernels_us"].items()})
PY
done
