#!/bin/bash
# Extra PMC passes on the bench (1 step) for the k_trace bottleneck analysis:
# issue/wait breakdown, TA (address unit) busy, L1/L2 hit behaviour.
export TMPDIR=/tmp
OUT=gpurun_out/prof2
rm -rf $OUT; mkdir -p $OUT
SCENE=${SCENE:-sphere_grid}
B="bench.py --scene $SCENE --no-cpu-baseline --steps 1 --warmup 0 --no-kernel-timing"
i=0
DEFAULT_GROUPS=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
  "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum" \
  "TCP_TOTAL_CACHE_ACCESSES_sum" "TCP_TCC_READ_REQ_sum" "TCP_TCP_LATENCY_sum" "TCC_HIT_sum TCC_MISS_sum" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES")
# PMC_GROUPS="A B;C D" overrides (groups separated by ';')
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -r -a GROUPS_ <<< "$PMC_GROUPS"; else GROUPS_=("${DEFAULT_GROUPS[@]}"); fi
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo profile_trace ok
