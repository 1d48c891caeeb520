#!/bin/bash
# PMC comparison of option sets (MASSRT_OPTIONS) on one scene (1 bench step each):
# TA busy / wavefronts, TCP accesses, LDS and VMEM instruction counts.
#   SCENE=sphere_grid CONFIGS="base:MASSRT_OPTIONS=treelet_kb=0;tl:MASSRT_OPTIONS=treelet_kb=16" bash tools/pmc_ab.sh
set -o pipefail
export TMPDIR=/tmp
SCENE=${SCENE:-sphere_grid}
OUT=gpurun_out/pmcab
mkdir -p $OUT
IFS=';' read -r -a CFGS <<< "$CONFIGS"
for c in "${CFGS[@]}"; do
  label=${c%%:*}; envs=${c#*:}
  for grp in "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_WAVES"; do
    tag=$(echo $grp | cut -c1-6)
    env $envs timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/${label}_$tag -o run --output-format csv -- \
      python3 bench.py --scene $SCENE --secondary none --no-cpu-baseline --no-configs --no-dropin --steps 1 --warmup 1 --no-kernel-timing \
      > $OUT/${label}_$tag.log 2>&1 || { echo "pmc $label failed"; tail -5 $OUT/${label}_$tag.log; exit 1; }
  done
  echo "== $label ($envs)"
  python3 tools/pmc_table.py $OUT/${label}_TA_TA_ | grep -A12 "^k_trace$"
  python3 tools/pmc_table.py $OUT/${label}_SQ_INS | grep -A12 "^k_trace$"
done
