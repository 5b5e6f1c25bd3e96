#!/bin/bash
# On the GPU box: the counter list and the PMC calibration passes of tools/pmc_calib (built here:
#   hipcc --offload-arch=gfx950 -O3 -o tools/bin/pmc_calib tools/pmc_calib.hip)
#   -> gpurun_out/calib/counters.txt, gpurun_out/calib/<pass>/run_counter_collection.csv
R=/root/repo
O=$R/gpurun_out/calib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || exit $?
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- $R/tools/bin/pmc_calib \
    > $O/$name.log 2>&1
}
pass fetch FETCH_SIZE || exit $?
pass write WRITE_SIZE || exit $?
# raw memory-side request counters, when this build lists them (one TCC group per pass)
for c in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B TCC_EA0_WRREQ TCC_EA0_WRREQ_64B \
         TCC_BUBBLE TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM; do
  if grep -qw "${c}" $O/counters.txt; then pass raw_$c ${c}_sum || exit $?; fi
done
echo calib done
