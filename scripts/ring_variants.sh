#!/bin/bash
# Timing-experiment builds of the ring plan (never the product library): group_ring.hip compiled with RING_EXP_*
# macros and linked with the product objects into incubator-pinot_amd/pinot_amd/variants/<name>.so, loaded by the
# bench through PINOT_GPU_LIB. Usage: scripts/ring_variants.sh name:"-DMACRO=1 ..." ...
set -e
cd "$(dirname "$0")/../incubator-pinot_amd"
mkdir -p build/variants pinot_amd/variants
objs=$(ls build/*.o | grep -v group_ring.o)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc -I/opt/rocm/include $flags \
    -c csrc/group_ring.hip -o build/variants/group_ring_$name.o &
done
wait
for spec in "$@"; do
  name=${spec%%:*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o pinot_amd/variants/$name.so $objs build/variants/group_ring_$name.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  echo "built pinot_amd/variants/$name.so"
done
