"""Summarises rocprofv3 --pmc passes over bench.py (tools/pmc_record.sh)
into the counters of the timed k_pipeline launch (the last dispatch of the
kernel: the warm-up call's launch comes first), per launch and per
macroblock, stamped with the SHA-256 of the library that ran and of its
code sections (JSON on stdout).

Units and corrections (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles (the ratios between them are unit-free);
FETCH_SIZE / WRITE_SIZE are KiB.  FETCH_SIZE is TCC_EA0_RDREQ x 64 B and is
doubled: calibrated in round 6 (tools/fetch_calib.hip,
profiles/r06_fetch_write_calib.log) for this kernel's own pattern -- a
4-lane quad gathering 8 bytes per lane from rows of a 2048-byte-stride
plane -- as for streaming reads, every L2 miss is one 128-byte request
(TCC_EA0_RDREQ_128B) tallied at 64 B.  WRITE_SIZE is exact: 64-byte
requests for whole-sector streaming stores, one 32-byte request per 16- or
4-byte partial store, each counted at its size.  Infinity-Cache hits are
counted, not excluded.  With the request-size passes (pmc_record.sh) the
reads are also given as TCC_EA0_RDREQ_128B x 128 + the rest x 64 and the
writes split into 64-byte / other requests and into IO (host-memory) and
atomic requests.

  python tools/pmc_summary.py --warmup W --steps S DIR [DIR ...]
"""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hartallo_amd import _lib  # noqa: E402  (code_sha256 only: loads no library)


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
        "kernel": "k_pipeline", "lib_sha256": hashlib.sha256(open(a.lib, "rb").read()).hexdigest(), "code_sha256": _lib.code_sha256(a.lib),
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
    out["fetch_size_factor"] = {"factor": 2.0, "calibrated": "round 6, tools/fetch_calib.hip: streaming 16 B/lane, the search's "
                                "8-byte quad gathers and 4-byte line reads all issue one 128-B request per L2 miss "
                                "(TCC_EA0_RDREQ_128B), FETCH_SIZE = requests x 64 B", "log": "profiles/r06_fetch_write_calib.log"}
    if "TCC_EA0_RDREQ_sum" in c and "TCC_EA0_RDREQ_128B_sum" in c:
        r128, rall = c["TCC_EA0_RDREQ_128B_sum"], c["TCC_EA0_RDREQ_sum"]
        out["read_requests_per_mb"] = {"all": round(rall / mbs, 1), "128B": round(r128 / mbs, 1),
                                       "bytes_per_mb": round((r128 * 128 + (rall - r128) * 64) / mbs, 1)}
    if "TCC_EA0_WRREQ_sum" in c and "TCC_EA0_WRREQ_64B_sum" in c:
        w64, wall = c["TCC_EA0_WRREQ_64B_sum"], c["TCC_EA0_WRREQ_sum"]
        out["write_requests_per_mb"] = {"all": round(wall / mbs, 1), "64B": round(w64 / mbs, 1), "32B_or_less": round((wall - w64) / mbs, 1),
                                        "bytes_per_mb": round((w64 * 64 + (wall - w64) * 32) / mbs, 1)}
        for k, n in (("TCC_EA0_WRREQ_WRITE_IO_32B_sum", "io_32B"), ("TCC_EA0_WRREQ_ATOMIC_DRAM_sum", "atomic_dram"),
                     ("TCC_EA0_WRREQ_WRITE_DRAM_sum", "write_dram")):
            if k in c:
                out["write_requests_per_mb"][n] = round(c[k] / mbs, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
