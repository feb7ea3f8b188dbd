"""Per-dispatch counter table of tools/fetch_calib runs (rocprofv3 csv files
of several passes).  Development tool: python tools/fetch_calib_summary.py csv..."""
import collections
import csv
import sys

agg = collections.defaultdict(float)
names = {}
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        agg[(d, r["Counter_Name"])] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"].split("(")[0]
cols = sorted({c for _, c in agg})
print("dispatch kernel " + " ".join(cols))
for d in sorted(names):
    if names[d].startswith("__amd"):
        continue
    print(d, names[d], " ".join(f"{agg.get((d, c), float('nan')):.0f}" for c in cols))
