#!/bin/bash
# rocprofv3 evidence for one bench scene: kernel-trace stats, then PMC counters
# in their own passes (FETCH_SIZE and WRITE_SIZE each alone; no --pmc together
# with trace domains). Summary -> profiles/pmc_<scene>.json, stamped with the
# config and the source hash so bench.py uses it only for the code it measured.
#   SCENE=mesh_ply bash tools/profile.sh
set -o pipefail
export TMPDIR=/tmp
SCENE=${SCENE:-sphere_grid}
TAG=${TAG:-}   # e.g. TAG=_solo with MASSRT_OPTIONS=queues=1: profiles/pmc_<scene>_solo.json
OUT=gpurun_out/prof_$SCENE$TAG
rm -rf $OUT; mkdir -p $OUT
# BENCH_EXTRA: the config's own size, e.g. "--width 3840 --height 2160 --spp-per-step 256" (config 5)
B="bench.py --scene $SCENE --no-cpu-baseline --no-dropin --no-configs --secondary none $BENCH_EXTRA"
P="--steps 1 --warmup 1 --no-kernel-timing"
run() {  # name, timeout, rocprofv3 args...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- python3 $B $EXTRA > $OUT/$name.log 2>&1
}
EXTRA="--steps 4 --warmup 1" run trace 300 --kernel-trace --stats && \
EXTRA="$P" run fetch 240 --pmc FETCH_SIZE && \
EXTRA="$P" run write 240 --pmc WRITE_SIZE && \
EXTRA="$P" run units 240 --pmc TA_TA_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum && \
EXTRA="$P" run sq 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES && \
EXTRA="$P" run sq2 240 --pmc SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
rc=$?
echo "profile $SCENE rc=$rc"
[ $rc -eq 0 ] && PMC_TAG=$TAG python3 tools/pmc_summary.py $OUT $SCENE > $OUT/summary.log 2>&1; tail -40 $OUT/summary.log
exit $rc
