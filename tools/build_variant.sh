#!/bin/bash
# Build an A/B variant of libmitsuba_hip.so with extra compile flags into
# gpurun_exp/lib_<name>.so (own object dir; the in-tree library is untouched).
# usage: tools/build_variant.sh <name> [extra hipcc flags...]   then MH_LIB=gpurun_exp/lib_<name>.so
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OBJ=/tmp/mh_variant_$NAME
mkdir -p "$OBJ" "$ROOT/gpurun_exp"
cd "$ROOT/mitsuba3-nasa_amd/csrc"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-fast-math -Wno-unused-function $*"
for f in mh_api.hip mh_kernels.hip mh_volwave.hip; do /opt/rocm/bin/hipcc $FLAGS -c $f -o "$OBJ/${f%.hip}.o" & done
/opt/rocm/bin/hipcc $FLAGS -fno-slp-vectorize -c mh_wavefront.hip -o "$OBJ/mh_wavefront.o" &  # as the Makefile
/opt/rocm/bin/hipcc $FLAGS -x hip -c mh_bvh.cpp -o "$OBJ/mh_bvh.o" &
/opt/rocm/bin/hipcc $FLAGS -x hip -c mh_comm.cpp -o "$OBJ/mh_comm.o" &
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/gpurun_exp/lib_$NAME.so" "$OBJ"/*.o -L/opt/rocm/lib -lrocprofiler-sdk-roctx -ldl -Wl,-rpath,/opt/rocm/lib
echo "$*" > "$ROOT/gpurun_exp/$NAME.flags"
echo "built gpurun_exp/lib_$NAME.so"
