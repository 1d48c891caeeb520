#!/bin/bash
# Round 6: SQ counters of k_trace on mesh_ply for the near-first walk (product
# and zero-margin probe) and the reference walk — VALU instructions and busy
# cycles per launch, to tell issue-bound from latency-bound.
set -o pipefail
export TMPDIR=/tmp
L=mass-raytrace_amd/massrt
B="bench.py --scene mesh_ply --no-cpu-baseline --no-dropin --no-configs --secondary none --steps 1 --warmup 1 --no-kernel-timing"
one() {  # name, env..., then counters after --
  local name=$1; shift
  mkdir -p gpurun_out/pmcw/$name
  env "$@" timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES \
    -d gpurun_out/pmcw/$name -o run --output-format csv -- python3 $B > gpurun_out/pmcw/$name.log 2>&1
}
two() {
  local name=$1; shift
  mkdir -p gpurun_out/pmcw/${name}_b
  env "$@" timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE \
    -d gpurun_out/pmcw/${name}_b -o run --output-format csv -- python3 $B > gpurun_out/pmcw/${name}_b.log 2>&1
}
one nf MASSRT_OPTIONS=traversal=1 && two nf MASSRT_OPTIONS=traversal=1 &&
one zr MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1 && two zr MASSRT_LIB=$L/libmassrt_zr.so MASSRT_OPTIONS=traversal=1 &&
one ref MASSRT_OPTIONS=traversal=0 && two ref MASSRT_OPTIONS=traversal=0
rc=$?
python3 tools/pmc_walks.py gpurun_out/pmcw || true
exit $rc
