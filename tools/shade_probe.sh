#!/bin/bash
# k_shade's HBM traffic split: FETCH_SIZE and WRITE_SIZE
# of the product library and of a probe build whose k_shade skips the
# scattered 16-B results[g] stores (wrong images; measurement only), one
# bench step of SCENE each, every pass its own rocprofv3 run.
#   make -C mass-raytrace_amd OUT=massrt/libmassrt_probe.so BUILD=build_probe EXTRA=-DMRT_PROBE_NO_RESULTS massrt/libmassrt_probe.so
#   SCENE=sphere_grid bash tools/shade_probe.sh
set -o pipefail
export TMPDIR=/tmp
SCENE=${SCENE:-sphere_grid}
OUT=gpurun_out/shade_probe_$SCENE
rm -rf $OUT; mkdir -p $OUT
B="bench.py --scene $SCENE --no-cpu-baseline --no-dropin --no-configs --secondary none --steps 1 --warmup 1 --no-kernel-timing"
for lib in libmassrt libmassrt_probe; do
  for pmc in FETCH_SIZE WRITE_SIZE; do
    MASSRT_LIB=mass-raytrace_amd/massrt/$lib.so timeout -k 10 240 rocprofv3 --pmc $pmc -d $OUT/${lib}_$pmc -o run \
      --output-format csv -- python3 $B > $OUT/${lib}_$pmc.log 2>&1 || { echo "FAILED $lib $pmc"; exit 1; }
    echo "done $lib $pmc"
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for lib in ("libmassrt", "libmassrt_probe"):
    row = {}
    for pmc in ("FETCH_SIZE", "WRITE_SIZE"):
        tot, n = collections.defaultdict(float), collections.defaultdict(set)
        for f in glob.glob(f"{out}/{lib}_{pmc}/**/run_counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                k = "k_shade" if "k_shade<false" in name else ("k_trace" if "k_trace<false" in name else "other")
                tot[k] += float(r["Counter_Value"])
                n[k].add(r["Dispatch_Id"])
        row[pmc] = {k: tot[k] / max(len(n[k]), 1) for k in tot}
    ks = row["FETCH_SIZE"].get("k_shade", 0.0) * 1024, row["WRITE_SIZE"].get("k_shade", 0.0) * 1024
    print(f"{lib}: k_shade per launch: FETCH_SIZE {ks[0] / 1e9:.3f} GB (x2 corrected {2 * ks[0] / 1e9:.3f}), WRITE_SIZE {ks[1] / 1e9:.3f} GB")
PY
