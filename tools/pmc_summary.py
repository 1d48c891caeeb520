"""Summarise rocprofv3 CSV output of tools/profile.sh into
profiles/pmc_<scene>.json (+ a printable table).

HBM bytes per k_trace launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024:
FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes
of wide (16 B/lane) reads (MI355X_MICROARCH.md §HBM), hence the x2.
"""
import csv
import glob
import json
import sys
from collections import defaultdict
from pathlib import Path

out_dir = Path(sys.argv[1])
scene = sys.argv[2] if len(sys.argv) > 2 else "sphere_grid"
REPO = Path(__file__).resolve().parents[1]


def rows(pattern):
    for f in glob.glob(str(out_dir / pattern), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    for k in ("k_trace_rays", "k_trace", "k_shade", "k_generate", "k_accumulate"):
        if k in name:
            return k + ("[counting]" if f"{k}<true" in name else "")
    return name[:40]


summary = {"scene": scene, "width": 1920, "height": 1080, "kernels": {}}
stats = list(rows("trace/**/*kernel_stats.csv"))
for r in stats:
    name = short(r.get("Name", r.get("KernelName", "")))
    summary["kernels"].setdefault(name, {})
    summary["kernels"][name].update({  # kernel-trace run
        "calls": int(r.get("Calls", 0)), "total_ns": float(r.get("TotalDurationNs", 0)),
        "avg_ns": float(r.get("AverageNs", 0)), "percent": float(r.get("Percentage", 0)),
    })

agg = defaultdict(lambda: defaultdict(list))
for sub in ("fetch", "write", "sq"):
    for r in rows(f"{sub}/**/*counter_collection.csv"):
        name = short(r.get("Kernel_Name", r.get("Kernel-Name", r.get("KernelName", ""))))
        cname = r.get("Counter_Name", r.get("Counter-Name", ""))
        try:
            val = float(r.get("Counter_Value", r.get("Counter-Value", 0)))
        except ValueError:
            continue
        did = r.get("Dispatch_Id", r.get("Dispatch-Id", ""))
        agg[name][cname].append((did, val))

for name, counters in agg.items():
    k = summary["kernels"].setdefault(name, {})
    for cname, vals in counters.items():
        per = defaultdict(float)
        for did, v in vals:
            per[did] += v  # sum over dimensions/instances within a dispatch
        k[f"{cname}_per_launch"] = sum(per.values()) / max(len(per), 1)
        k[f"{cname}_launches"] = len(per)

t = summary["kernels"].get("k_trace", {})
if "FETCH_SIZE_per_launch" in t and "WRITE_SIZE_per_launch" in t:
    t["hbm_bytes_per_launch"] = (2 * t["FETCH_SIZE_per_launch"] + t["WRITE_SIZE_per_launch"]) * 1024
    summary["k_trace_hbm_bytes_per_launch"] = t["hbm_bytes_per_launch"]
if "SQ_INSTS_VALU_per_launch" in t and "SQ_WAVES_per_launch" in t:
    t["valu_insts_per_wave"] = t["SQ_INSTS_VALU_per_launch"] / max(t["SQ_WAVES_per_launch"], 1)

print(json.dumps(summary, indent=1))
dst = REPO / "profiles" / f"pmc_{scene}.json"
dst.write_text(json.dumps(summary, indent=1))
print("wrote", dst)
