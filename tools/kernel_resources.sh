#!/bin/bash
# VGPRs / scratch / occupancy per kernel of render.hip (compiler remarks; no GPU needed).
cd "$(dirname "$0")/../mass-raytrace_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -mllvm -simplifycfg-sink-common=false -Wno-unused-function -Wno-unused-value \
  --offload-device-only -Rpass-analysis=kernel-resource-usage $KR_EXTRA -c csrc/device/render.hip -o /tmp/kr.o 2>&1 |
  sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name:/{n=$NF} /VGPRs:/{v=$NF} /ScratchSize/{sc=$NF} /Occupancy/{print n, "vgpr", v, "scratch", sc, "occ", $NF}' |
  c++filt | sed -e 's/(anonymous namespace):://g' -e 's/(mrt::DevScene.*)//' -e 's/(mrt::.*)//'
