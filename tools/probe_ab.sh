#!/bin/bash
# Per-kernel probe times of library variants in one box session (TGN wiki step, graph replay + eager probes):
#   tools/probe_ab.sh <tag> <variant> ...   variant = default | build_var/<name> (a libtgnx.so dir) |
#   build_var/<tree> holding its own bench.py (an older tree)  ->  gpurun_out/<tag>_probe_ab.txt
tag=$1; shift
R=/root/repo
out=$R/gpurun_out/${tag}_probe_ab.txt
: > $out
for round in 1 2; do
  for v in "$@"; do
    unset TGNX_LIB; b=$R/bench.py
    if [ "$v" != default ]; then
      if [ -f $R/$v/bench.py ]; then b=$R/$v/bench.py; else export TGNX_LIB=$R/$v/libtgnx.so; fi
    fi
    r=$(timeout -k 10 300 python $b --model ${MODEL:-tgn} --only --steps 300 --warmup 30 \
        --no-cpu-baseline ${EXTRA} 2>/dev/null | grep metric) || exit 1
    echo "$v $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], {k: round(x, 1) for k, x in d["kernels_us"].items()})')" >> $out
  done
done
cat $out
