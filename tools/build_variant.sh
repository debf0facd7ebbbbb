#!/bin/bash
# A/B variant of libgrace_hip that differs only in one source's compile-time knobs: recompiles
# grace_amd/csrc/SRC with the given -D defines and links it with the default build's other objects.
#   tools/build_variant.sh SRC NAME "DEF1=V1 DEF2=V2"  ->  grace_amd/lib/libgrace_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
src=$1; name=$2; defs=""
for d in $3; do defs="$defs -D$d"; done
obj=grace_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
    -Wno-unused-function $defs -c grace_amd/csrc/$src -o /tmp/${src}_$name.o
others=$(ls $obj/*.o | grep -v "/$src.o\$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others /tmp/${src}_$name.o -o grace_amd/lib/libgrace_hip_$name.so
echo grace_amd/lib/libgrace_hip_$name.so
