#!/bin/bash
# Build an A/B variant of the library with extra defines (CPU side, before a gpurun call):
#   tools/build_variant.sh <suffix> [-DFLAG ...]  ->  fleetflow_amd/libfleetplace<suffix>.so
set -e
cd "$(dirname "$0")/../fleetflow_amd/csrc"
suffix=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics "$@" \
  -shared -o ../libfleetplace$suffix.so fp_ctx.hip fp_place.hip fp_pipe.hip fp_order.hip fp_feas.hip fp_gen.hip fp_small.hip
