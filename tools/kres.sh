#!/bin/bash
# per-kernel resource summary: tools/kres.sh file.hip [regex]
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -c "$1" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed -n 's/.*remark: //p' | sed 's/ \[-Rpass.*//' | awk '
/Function Name/ {name=$3} /VGPRs:/ {v=$2} /SGPRs Spill/ {ss=$3} /ScratchSize/ {sc=$3} /Occupancy/ {occ=$3}
/LDS Size/ {print name, "vgpr="v, "sgpr_spill="ss, "scratch="sc, "occ="occ, "lds="$5}' | c++filt | grep -E "${2:-.}"
