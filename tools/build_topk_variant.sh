#!/bin/bash
# A/B variant of libgrace_hip that differs only in csrc/topk.hip's compile-time knobs: recompiles
# topk.hip with the given -D defines and links it with the default build's other objects.
#   tools/build_topk_variant.sh NAME "DEF1=V1 DEF2=V2"  ->  grace_amd/lib/libgrace_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
name=$1; defs=""
for d in $2; do defs="$defs -D$d"; done
obj=grace_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt \
    -Wno-unused-function $defs -c grace_amd/csrc/topk.hip -o /tmp/topk_$name.o
others=$(ls $obj/*.o | grep -v '/topk.hip.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others /tmp/topk_$name.o -o grace_amd/lib/libgrace_hip_$name.so
echo grace_amd/lib/libgrace_hip_$name.so
