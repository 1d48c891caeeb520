#!/bin/bash
# Copy a final-evidence call's outputs (gpurun_out/) into profiles/: stamped
# PMC summaries, kernel stats and profile summaries of the named profile
# directories, and the suite/smoke logs when present.
cd "$(dirname "$0")/.."
for name in "$@"; do
  d=gpurun_out/prof_$name
  cp $d/pmc_*.json profiles/ &&
  cp $d/trace/run_kernel_stats.csv profiles/r6_${name}_kernel_stats.csv &&
  cp $d/summary.log profiles/r6_profile_logs/prof_$name.summary.log || exit 1
done
[ -s gpurun_out/session/pytest_gpu.log ] && cp gpurun_out/session/pytest_gpu.log profiles/r6_pytest_gpu.log
[ -s gpurun_out/session/smoke.log ] && cp gpurun_out/session/smoke.log profiles/r6_smoke.log
exit 0
