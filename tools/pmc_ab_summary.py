"""Per-launch counter totals of the last k_pipeline dispatch of every pass
of tools/pmc_ab.sh.  python tools/pmc_ab_summary.py gpurun_out/pmcab_<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    for d in sorted(glob.glob(os.path.join(root, "l*_*"))):
        if not os.path.isdir(d):
            continue
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            continue
        per = defaultdict(lambda: defaultdict(float))
        for row in csv.DictReader(open(files[0])):
            if "k_pipeline" not in row.get("Kernel_Name", ""):
                continue
            per[int(row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
        if not per:
            continue
        last = per[max(per)]
        print(os.path.basename(d), " ".join(f"{k}={v:.4g}" for k, v in sorted(last.items())))


if __name__ == "__main__":
    main()
