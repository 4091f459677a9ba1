#!/bin/bash
# Per-kernel VGPR / AGPR / scratch / occupancy of a HIP source (gfx950), e.g.
#   tools/regs.sh cnn-super-resolution_amd/csrc/hip/train_fused.hip [-DFLAG ...]
src=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I$R/include -I$R/cnn-super-resolution_amd/csrc/hip \
  "$@" -x hip -c "$src" -o /tmp/regs_$$.o --cuda-device-only -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -E 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name:/{n=$NF} / VGPRs: /{v=$NF} /AGPRs: /{a=$NF} /ScratchSize/{sc=$NF} /Occupancy/{print substr(n,1,90), "vgpr=" v, "agpr=" a, "scratch=" sc, "occ=" $NF}'
rm -f /tmp/regs_$$.o
