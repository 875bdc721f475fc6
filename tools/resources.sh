#!/bin/bash
# Per-kernel VGPR / spill / occupancy table from the compiler's resource remarks.
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-value -Wno-unused-result -I include $RES_DEFS \
  -c trpo-robot-control_amd/csrc/trpo_kernels.hip -o /tmp/_res.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  sed -n 's/.*remark: *//p' | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/{n=$3} /^VGPRs:/{v=$2} /^AGPRs:/{a=$2} /Occupancy/{o=$4} /VGPRs Spill/{sp=$3} /LDS Size/{print n, "vgpr="v, "agpr="a, "occ="o, "spill="sp}' |
  c++filt | sed 's/(.*)//' | grep "${1:-.}"
