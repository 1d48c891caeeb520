"""Summarise tools/profile.sh output into profiles/pmc_<scene>.json.

Per kernel: rocprofv3 kernel-trace stats (calls, average duration) and the
PMC counters of the profiled step, summed over the dimensions of a dispatch
and averaged over dispatches. Derived for k_trace:
  hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (KiB counters;
      gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane reads,
      MI355X_MICROARCH.md §HBM)
  ta_busy   = TA_TA_BUSY_sum / (GRBM_GUI_ACTIVE/8 XCDs) / CUs   (address unit)
  l1_hit    = 1 - TCP_TCC_READ_REQ_sum / TCP_TOTAL_CACHE_ACCESSES_sum
  l2_hit    = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES
  valu_busy = 2 * SQ_INSTS_VALU / (GRBM_GUI_ACTIVE/8) / (4 SIMDs x CUs)
              (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles)
  lds_busy  = SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE/8) / CUs
The stamp (scene, size, spp per step, source hash) ties the file to the code
and configuration it measured; bench.py ignores a file whose stamp differs.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
out_dir = Path(sys.argv[1])
scene = sys.argv[2] if len(sys.argv) > 2 else "sphere_grid"


def traced_config():
    """(width, height, spp per step, walk) of the bench line the trace run
    printed (walk: the traversal the context took, MRT_TRAVERSAL_*)."""
    lines = (out_dir / "trace.log").read_text().splitlines() if (out_dir / "trace.log").exists() else []
    for ln in reversed(lines):
        if ln.startswith("{"):
            c = json.loads(ln)["config"]
            return c["width"], c["height"], c["spp_per_step"], int(c.get("tuning", {}).get("traversal", 0))
    raise SystemExit(f"no bench line in {out_dir / 'trace.log'}: pass W H SPP TRAVERSAL")


W, H, SPP, TRAV = (int(x) for x in sys.argv[3:7]) if len(sys.argv) > 6 else traced_config()
N_CU, N_XCD = 256, 8


def rows(pattern):
    for f in glob.glob(str(out_dir / pattern), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def short(name):
    for k in ("k_trace_rays", "k_trace", "k_shade", "k_generate", "k_accumulate", "k_shard_pack", "k_shard_unpack"):
        if k in name:
            return k + ("[counting]" if f"{k}<true" in name else "")
    return name[:40]


import bench  # noqa: E402  (source hash of the library the profile measured)

summary = {"scene": scene, "width": W, "height": H,
           "stamp": {"scene": scene, "width": W, "height": H, "spp_per_step": SPP, "src": bench.src_hash(),
                     # the walk profiled, as the bench line reports it (AUTO resolved per scene)
                     "traversal": TRAV},
           "kernels": {}}
for r in rows("trace/**/*kernel_stats.csv"):
    name = short(r.get("Name", r.get("KernelName", "")))
    k = summary["kernels"].setdefault(name, {})
    k.update({"calls": int(r.get("Calls", 0)), "total_ns": float(r.get("TotalDurationNs", 0)),
              "avg_ns": float(r.get("AverageNs", 0)), "percent": float(r.get("Percentage", 0))})
    k["kernel_name"] = r.get("Name", r.get("KernelName", ""))[:160]

agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for sub in ("fetch", "write", "units", "sq", "sq2"):
    for r in rows(f"{sub}/**/*counter_collection.csv"):
        name = short(r.get("Kernel_Name", r.get("Kernel-Name", r.get("KernelName", ""))))
        cname = r.get("Counter_Name", r.get("Counter-Name", ""))
        try:
            val = float(r.get("Counter_Value", r.get("Counter-Value", 0)))
        except ValueError:
            continue
        did = r.get("Dispatch_Id", r.get("Dispatch-Id", ""))
        agg[name][f"{sub}:{cname}"][did] += val  # sum over dimensions within a dispatch

for name, counters in agg.items():
    k = summary["kernels"].setdefault(name, {})
    for key, per in counters.items():
        cname = key.split(":", 1)[1]
        k[cname if cname != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE_{key.split(':')[0]}"] = \
            sum(per.values()) / max(len(per), 1)
        k.setdefault("pmc_launches", len(per))

for name, k in summary["kernels"].items():
    if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
        k["hbm_bytes_per_launch"] = (2 * k["FETCH_SIZE"] + k["WRITE_SIZE"]) * 1024
    g = k.get("GRBM_GUI_ACTIVE_units")
    if g and "TA_TA_BUSY_sum" in k:
        k["ta_busy"] = k["TA_TA_BUSY_sum"] / (g / N_XCD) / N_CU
    if k.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        k["l1_hit"] = 1 - k.get("TCP_TCC_READ_REQ_sum", 0) / k["TCP_TOTAL_CACHE_ACCESSES_sum"]
    if k.get("TCC_HIT_sum", 0) + k.get("TCC_MISS_sum", 0) > 0:
        k["l2_hit"] = k["TCC_HIT_sum"] / (k["TCC_HIT_sum"] + k["TCC_MISS_sum"])
    if k.get("SQ_WAVE_CYCLES"):
        k["wait_frac"] = k.get("SQ_WAIT_ANY", 0) / k["SQ_WAVE_CYCLES"]
    g2 = k.get("GRBM_GUI_ACTIVE_sq2")
    if g and "SQ_INSTS_VALU" in k:
        k["valu_busy"] = 2 * k["SQ_INSTS_VALU"] / (g / N_XCD) / (4 * N_CU)
    if g2 and "SQ_LDS_IDX_ACTIVE" in k:
        k["lds_busy"] = k["SQ_LDS_IDX_ACTIVE"] / (g2 / N_XCD) / N_CU
    if k.get("SQ_WAVES") and "SQ_INSTS_VALU" in k:
        k["valu_insts_per_wave"] = k["SQ_INSTS_VALU"] / k["SQ_WAVES"]

t = summary["kernels"].get("k_trace", {})
if "hbm_bytes_per_launch" in t:
    summary["k_trace_hbm_bytes_per_launch"] = t["hbm_bytes_per_launch"]
print(json.dumps(summary, indent=1))


# bench.py reads profiles/pmc_<scene>_nf.json for the near-first walk, pmc_<scene>_solo.json (PMC_TAG) alone
tag = os.environ.get("PMC_TAG", "") or ("_nf" if TRAV == 1 else "")
if tag:
    summary["tag"] = tag
    summary["options"] = os.environ.get("MASSRT_OPTIONS", "")
for dst in (REPO / "profiles" / f"pmc_{scene}{tag}.json", out_dir / f"pmc_{scene}{tag}.json"):  # out_dir: travels back
    dst.write_text(json.dumps(summary, indent=1))
    print("wrote", dst)
