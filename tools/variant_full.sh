#!/bin/bash
# Builds a whole-library timing variant (every source with extra flags, for
# macros the host side shares, e.g. DCP_MF_WAVES) into
# build/var/libdcp_<name>.so:  NAME=w2 FLAGS="-DDCP_MF_WAVES=2" bash tools/variant_full.sh
set -e
cd "$(dirname "$0")/../3d-dycoreplanet_amd"
mkdir -p build/var build/vfull_$NAME
objs=""
for f in $(grep -E "^(HOSTSRC|HIPSRC)" Makefile | sed 's/^[A-Z]*SRC *:= *//'); do
  o=build/vfull_$NAME/$(basename ${f%.*}).o
  if [[ $f == *.cpp ]]; then extra=-fopenmp; else extra=-munsafe-fp-atomics; fi
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 $extra $FLAGS -c $f -o $o &
  objs="$objs $o"
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
/opt/rocm/bin/hipcc -shared -fopenmp --offload-arch=gfx950 -o build/var/libdcp_$NAME.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf build/vfull_$NAME
