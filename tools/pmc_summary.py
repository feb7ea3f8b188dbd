"""Summarises rocprofv3 --pmc passes over bench.py (tools/pmc_record.sh)
into the counters of the timed k_pipeline launch (the last dispatch of the
kernel: the warm-up call's launch comes first), per launch and per
macroblock, stamped with the SHA-256 of the library that ran (JSON on
stdout).

Units and corrections (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles (the ratios between them are unit-free);
FETCH_SIZE / WRITE_SIZE are KiB (TCC_EA0_*REQ x 64 B / 1024) and FETCH_SIZE
is doubled for gfx950 (128-B requests tallied at 64 B; calibrated for
16 B/lane streaming reads -- this kernel's byte gathers are uncalibrated, and
Infinity-Cache hits are counted, not excluded).

  python tools/pmc_summary.py --warmup W --steps S DIR [DIR ...]
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timed_launch(d):
    """{counter: value} of the last k_pipeline dispatch in one pass."""
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith("k_pipeline"):
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id") or r.get("Start_Timestamp")
        acc[int(key)][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc[max(acc)], len(acc)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--warmup", type=int, required=True)
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1088)
    ap.add_argument("--workgroups", type=int, default=0, help="k_pipeline workgroups (0: one per resident slot)")
    ap.add_argument("--streams-per-gpu", type=int, default=1)
    ap.add_argument("--lib", default=os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so"))
    ap.add_argument("dirs", nargs="+")
    a = ap.parse_args()
    c, launches = {}, set()
    for d in a.dirs:
        v, n = timed_launch(d)
        c.update(v)
        launches.add(n)
    mbs = a.steps * (a.width // 16) * (a.height // 16)  # the timed call: one launch of `steps` pictures
    out = {
        "kernel": "k_pipeline", "lib_sha256": hashlib.sha256(open(a.lib, "rb").read()).hexdigest(),
        "recorded": time.strftime("%Y-%m-%d"), "warmup": a.warmup, "steps": a.steps,
        # the workload the counters belong to (bench.py uses them only for this one)
        "width": a.width, "height": a.height, "workgroups": a.workgroups, "streams_per_gpu": a.streams_per_gpu,
        "k_pipeline_dispatches_per_pass": sorted(launches), "macroblocks_per_launch": mbs,
        "counters": {k: c[k] for k in sorted(c)},
    }
    if "SQ_WAVE_CYCLES" in c:
        out["sq_wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        out["sq_issue_frac"] = round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        out["valu_insts_per_mb"] = round(c["SQ_INSTS_VALU"] / mbs)
        out["lds_insts_per_mb"] = round(c["SQ_INSTS_LDS"] / mbs)
        out["salu_insts_per_mb"] = round(c["SQ_INSTS_SALU"] / mbs)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd, wr = 2.0 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        out.update({"fetch_bytes_per_launch_x2": rd, "write_bytes_per_launch": wr, "traffic_bytes_per_launch": rd + wr,
                    "fetch_bytes_per_mb_x2": round(rd / mbs, 1), "write_bytes_per_mb": round(wr / mbs, 1),
                    "traffic_bytes_per_mb": round((rd + wr) / mbs, 1)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
