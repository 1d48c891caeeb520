#!/bin/bash
# Round evidence on the current code: rocprofv3 kernel stats + PMC passes for
# the two bench scenes (profiles/pmc_<scene>.json, stamped), then the default
# bench line (headline sphere_grid + mesh_ply secondary + CPU baselines).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for sc in ${SCENES:-sphere_grid mesh_ply}; do
  SCENE=$sc bash tools/profile.sh > gpurun_out/profile_$sc.log 2>&1 || { echo "profile $sc failed"; tail -20 gpurun_out/profile_$sc.log; exit 1; }
  tail -3 gpurun_out/profile_$sc.log
done
cp profiles/pmc_*.json gpurun_out/ 2>/dev/null
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 900 python bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -c 400 gpurun_out/bench.log
