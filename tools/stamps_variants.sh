#!/bin/bash
# On the GPU box: stamps timeline of each var/<name>/libtgnx.so -> gpurun_out/<tag>_<name>.txt, summary on stdout
tag=${1:-sv}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in var/*/; do
  n=$(basename $d)
  TGNX_LIB=$PWD/$d/libtgnx.so timeout -k 10 200 python tools/stamps.py --steps 20 --bins ${STAMPS_ARGS} > gpurun_out/${tag}_$n.txt 2>&1 || { echo "variant $n failed"; tail -5 gpurun_out/${tag}_$n.txt; exit 1; }
  echo "== $n"; sed -n '4,16p' gpurun_out/${tag}_$n.txt; grep -E "^sum of spans|checkpoints" gpurun_out/${tag}_$n.txt
done
