#!/bin/bash
# Build libtgnx.so variants of tgnx_tgnn.hip with extra -D flags for kernel-geometry timing
# experiments: tools/build_variants.sh name "-DFOO=1 ..." [name "flags"]...  -> build_var/<name>/libtgnx.so
set -e
cd "$(dirname "$0")/../tgb-tgn-dgl_amd"
make -s -j8
OTHERS=$(ls build/*.o | grep -v tgnx_tgnn.o)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p ../build_var/$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result $flags \
    -c csrc/tgnx_tgnn.hip -o ../build_var/$name/tgnx_tgnn.o &
done
wait
for d in ../build_var/*/; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/libtgnx.so $d/tgnx_tgnn.o $OTHERS
done
