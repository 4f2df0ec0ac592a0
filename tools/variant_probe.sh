#!/bin/bash
# Builds timing variants of one kernel file into build/var/libdcp_<name>.so:
#   VARIANTS="base: b12:-DDCP_SCATTER_BATCH=12" [SRC=assembly] bash tools/variant_probe.sh
# (name:extra hipcc flags for kernels/$SRC.hip). Time them on the GPU box with
# python3 tools/variant_probe.py (assembly) or tools/mf_probe.py (matfree).
set -e
cd "$(dirname "$0")/../3d-dycoreplanet_amd"
make -s libdcp.so
mkdir -p build/var
SRC=${SRC:-assembly}
OTHERS=$(ls build/*.o | grep -v "/$SRC.o")
for spec in ${VARIANTS:-base:}; do
  name=${spec%%:*}; flags=${spec#*:}
  if [ -f csrc/$SRC.cpp ]; then srcf=csrc/$SRC.cpp; extra=-fopenmp; else srcf=csrc/kernels/$SRC.hip; extra=-munsafe-fp-atomics; fi
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 $extra ${flags//,/ } \
    -c $srcf -o build/var/${SRC}_$name.o
  /opt/rocm/bin/hipcc -shared -fopenmp --offload-arch=gfx950 -o build/var/libdcp_$name.so $OTHERS \
    build/var/${SRC}_$name.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
