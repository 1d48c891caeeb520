"""Per-kernel PMC table from tools/profile_trace.sh output (sums over the
dimensions of one dispatch, averaged over dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        for k in ("k_trace", "k_shade", "k_generate", "k_accumulate"):
            if k in name:
                name = k + ("[count]" if f"{k}<true" in name else "")
                break
        else:
            continue
        agg[name][r["Counter_Name"]][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
for name, cs in sorted(agg.items()):
    print(name)
    for c, per in sorted(cs.items()):
        print(f"   {c:40s} {sum(per.values()) / len(per):16.1f}  (n={len(per)})")
