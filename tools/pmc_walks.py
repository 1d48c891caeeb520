"""Per-launch SQ counters of k_trace from tools/r6_pmc_walks.sh (one line per walk)."""
import csv
import glob
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
for name in ("nf", "zr", "ref"):
    tot = defaultdict(float)
    launches = defaultdict(set)
    for sub in (name, name + "_b"):
        for f in glob.glob(str(root / sub / "**" / "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "k_trace" not in row.get("Kernel_Name", "") or "true" in row["Kernel_Name"].split("<")[1][:5]:
                    continue
                tot[row["Counter_Name"]] += float(row["Counter_Value"])
                launches[row["Counter_Name"]].add(row.get("Dispatch_Id", ""))
    if not tot:
        print(name, "no data")
        continue
    per = {k: v / max(1, len(launches[k])) for k, v in tot.items()}
    clk = per.get("GRBM_GUI_ACTIVE", 0) / 8
    s = f"{name:4s} launches {len(launches.get('SQ_INSTS_VALU', []))}  "
    s += "  ".join(f"{k} {v:.4g}" for k, v in sorted(per.items()))
    if clk:
        s += f"  | clk/launch {clk:.4g}  valu_busy {2 * per.get('SQ_INSTS_VALU', 0) / clk / 1024:.3f}"
        s += f"  active_valu/clk/simd {per.get('SQ_ACTIVE_INST_VALU', 0) * 4 / clk / 1024:.3f}"
    if per.get("SQ_INSTS_VALU") and per.get("SQ_WAVE_CYCLES"):
        s += f"  wait_frac {per.get('SQ_WAIT_ANY', 0) / per['SQ_WAVE_CYCLES']:.3f}"
    print(s)
