#!/bin/bash
# Print VGPR / scratch / occupancy of every kernel in kernels/decode.hip (gfx950 cross-compile).
cd "$(dirname "$0")/../parquet-go_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -Ikernels -c kernels/decode.hip \
  -o /tmp/pqh_ru.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{n=$3} /^VGPRs:/{v=$2} /ScratchSize/{s=$3} /Occupancy/{print n, "vgpr=" v, "scratch=" s, "occ=" $3}'
