#!/bin/bash
# A levelizer A/B build (CPU side, before a gpurun call): fp_order.hip with extra defines, linked
# with the production objects of every other translation unit (run make first).
#   tools/build_order_variant.sh <suffix> [-DFLAG ...]  ->  fleetflow_amd/libfleetplace<suffix>.so
set -e
cd "$(dirname "$0")/../fleetflow_amd/csrc"
suffix=$1; shift
mkdir -p build/ov$suffix
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics "$@" \
  -c fp_order.hip -o build/ov$suffix/fp_order.o
objs=$(ls build/*.o | grep -v '/fp_order.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libfleetplace$suffix.so build/ov$suffix/fp_order.o $objs
