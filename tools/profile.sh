#!/bin/bash
# rocprofv3 evidence for the bench config: kernel-trace stats, then PMC
# counters in their own passes (FETCH_SIZE and WRITE_SIZE cannot share a pass
# on gfx950; no --pmc together with trace domains).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/prof
rm -rf $OUT; mkdir -p $OUT
SCENE=${SCENE:-sphere_grid}
B="bench.py --scene $SCENE --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $B --steps 4 --warmup 1 > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --no-kernel-timing > $OUT/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --no-kernel-timing > $OUT/write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 $B --steps 1 --warmup 0 --no-kernel-timing > $OUT/sq.log 2>&1
rc=$?
echo "profile rc=$rc"
find $OUT -name "*.csv" | head -20
python3 tools/pmc_summary.py $OUT $SCENE > $OUT/summary.log 2>&1; cat $OUT/summary.log | tail -30
exit $rc
