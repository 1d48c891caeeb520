# Runs tools/debug_parity.py against each bisection build; stops at the first
# timeout/abort/segfault (no further GPU work after a failure of that kind).
mkdir -p gpurun_out
for L in $BIS_POINTS; do
  echo "== $L" >> gpurun_out/bis.log
  MASSRT_LIB=$PWD/mass-raytrace_amd/build_bis/libmassrt_b$L.so timeout -k 10 60 python tools/debug_parity.py model > gpurun_out/bis_$L.log 2>&1
  rc=$?
  grep "random\|persistent\|Error" gpurun_out/bis_$L.log >> gpurun_out/bis.log
  echo "rc $rc" >> gpurun_out/bis.log
  if [ $rc -ge 124 ]; then exit $rc; fi
done
