#!/bin/bash
# One parameterised GPU-box session (replaces round 1-2's one-off gpu_*.sh).
# Every GPU step has its own time limit; steps chain with && so the first
# failure (fault, abort, time limit) ends the session — no step is retried.
#
#   bash tools/gpu_session.sh tests                 # pytest -m gpu + smoke
#   bash tools/gpu_session.sh bench [bench args]    # the default bench line (+ args)
#   bash tools/gpu_session.sh profile SCENE...      # rocprofv3 stats + stamped PMC (tools/profile.sh)
#   bash tools/gpu_session.sh configs               # every BASELINE config scene, timing only
#   LABELS="a b" LIBS="x.so y.so" bash tools/gpu_session.sh ab   # bench per library build (MASSRT_LIB)
#   SWEEP=$'base\ntl MASSRT_OPTIONS=treelet_kb=16' bash tools/gpu_session.sh sweep   # bench per option set
#   bash tools/gpu_session.sh rehearse              # bench.py --gpus 2 --devices 0,0 (one process, peer gather)
# SCENES (default "sphere_grid mesh_ply") and STEPS (default 3) apply to ab / sweep / args;
# BENCH_ARGS (e.g. "--spp-per-step 1024") is appended to every sweep run.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/session
MODE=$1; shift
SCENES=${SCENES:-"sphere_grid mesh_ply"}
STEPS=${STEPS:-3}

line() {  # log, label: one summary line of a bench log
  python3 -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline'] or {}; s=j.get('roofline_k_shade') or {}
print('%-28s %-12s %8.1f Msamples/s  %8.1f ms/step  k_trace %.3f ms  k_shade %.3f ms  util %.3f' % (sys.argv[2], j['config']['scene'], j['value'], j['ms_per_step'], r.get('avg_launch_ms', 0), s.get('avg_launch_ms', 0), r.get('lane_utilisation', 0)))" "$1" "$2"
}
quick() {  # label, log, bench args...: a timing-only bench of one scene
  local label=$1 log=$2; shift 2
  timeout -k 10 400 python bench.py --secondary none --no-cpu-baseline --no-dropin --no-configs "$@" > $log 2>&1 || { echo "FAILED $label"; tail -5 $log; return 1; }
  line $log $label
}

case $MODE in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/session/pytest_gpu.log 2>&1 && tail -1 gpurun_out/session/pytest_gpu.log &&
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/session/smoke.log 2>&1 &&
    tail -1 gpurun_out/session/smoke.log ;;
  bench)
    timeout -k 10 900 python -u bench.py "$@" > gpurun_out/session/bench.log 2> gpurun_out/session/bench.err &&
    line gpurun_out/session/bench.log headline ;;
  profile)
    for sc in "$@"; do SCENE=$sc bash tools/profile.sh > gpurun_out/session/profile_$sc.log 2>&1 || exit 1; done ;;
  configs)
    quick c2_sphere_grid gpurun_out/session/c2.log --scene sphere_grid --steps 2 &&
    quick c3_cube_field gpurun_out/session/c3.log --scene cube_field --steps 1 &&
    quick c4_mesh_ply gpurun_out/session/c4p.log --scene mesh_ply --steps 2 &&
    quick c4_mesh_obj gpurun_out/session/c4o.log --scene mesh_obj --steps 2 &&
    quick c5_mesh_obj_textured_4k gpurun_out/session/c5.log --scene mesh_obj_textured --width 3840 --height 2160 \
      --spp-per-step 256 --total-spp 4096 --steps 2 &&
    quick menger gpurun_out/session/menger.log --scene menger --spp-per-step 256 --steps 1 ;;
  ab)
    set -- $LIBS; labels=($LABELS); k=0
    for lib in "$@"; do
      lab=${labels[$k]:-$(basename $lib .so)}; k=$((k + 1))
      for sc in $SCENES; do
        MASSRT_LIB=$lib quick "$lab" gpurun_out/session/ab_${lab}_$sc.log --scene $sc --steps $STEPS $BENCH_ARGS || exit 1
      done
    done ;;
  sweep)
    while IFS= read -r cfg; do
      [ -z "$cfg" ] && continue
      set -- $cfg; lab=$1; shift
      for sc in $SCENES; do
        log=gpurun_out/session/sweep_${lab}_$sc.log
        env "$@" timeout -k 10 400 python bench.py --scene $sc --secondary none --no-cpu-baseline --no-dropin --no-configs \
          --steps $STEPS $BENCH_ARGS > $log 2>&1 || { echo "FAILED $lab $sc"; tail -5 $log; exit 1; }
        line $log $lab
      done
    done <<< "$SWEEP" ;;
  args)  # ARGSETS=$'s256 --spp-per-step 256\ns1k --spp-per-step 1024 --steps 1': bench per argument set
    while IFS= read -r cfg; do
      [ -z "$cfg" ] && continue
      set -- $cfg; lab=$1; shift
      for sc in $SCENES; do
        quick "$lab" gpurun_out/session/args_${lab}_$sc.log --scene $sc --steps $STEPS "$@" || exit 1
      done
    done <<< "$ARGSETS" ;;
  rehearse)  # N=2 on the 1-GPU box: one process, one context over devices {0,0}, peer-copy gather
    timeout -k 10 600 python -u bench.py --gpus 2 --devices 0,0 --steps 2 --secondary none --no-cpu-baseline \
      --no-dropin --no-configs > gpurun_out/session/rehearse2.log 2>&1 &&
    tail -1 gpurun_out/session/rehearse2.log | cut -c1-600 ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
