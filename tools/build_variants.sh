#!/bin/bash
# Build libtgnx.so variants with extra -D flags for kernel-geometry timing experiments:
#   tools/build_variants.sh name "-DFOO=1 ..." [name "flags"]...  -> build_var/<name>/libtgnx.so
#   (OUT=var: into var/<name>/ instead, which travels to the GPU box)
# (every csrc/*.hip recompiled with the flags; select one at run time with TGNX_LIB=...)
set -e
cd "$(dirname "$0")/../tgb-tgn-dgl_amd"
make -s -j8
# (only the named variants are rebuilt; others in build_var/ are kept)
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2; BUILT="$BUILT ../${OUT:-build_var}/$name/"
  rm -rf ../${OUT:-build_var}/$name; mkdir -p ../${OUT:-build_var}/$name
  for src in csrc/*.hip; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result $flags \
      -c $src -o ../${OUT:-build_var}/$name/$(basename $src .hip).o &
  done
  cp build/tgnx_host.o ../${OUT:-build_var}/$name/
done
wait
for d in $BUILT; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $d/libtgnx.so $d/*.o
done
