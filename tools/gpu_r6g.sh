#!/bin/bash
# stamps timeline of the wiki-shaped TGN step (stamps build), the last-ending workgroups per launch
set -o pipefail
cd /root/repo
mkdir -p gpurun_out
T=${1:-r6g}
TGNX_LIB=/root/repo/var/stamps/libtgnx.so timeout -k 10 300 python tools/stamps.py --steps 20 --top 6 > gpurun_out/${T}_stamps_top.txt 2>&1 || { tail -20 gpurun_out/${T}_stamps_top.txt; exit 1; }
cat gpurun_out/${T}_stamps_top.txt
