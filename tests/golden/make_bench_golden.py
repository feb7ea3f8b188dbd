"""Per-frame MD5s of the reference encoder's output for the BASELINE-sized
workloads (tests/golden/bench_golden.json).

The streams themselves are too large to commit, so each workload is encoded
by oracle/_ref/ref_enc (the reference's own C sources, driven through
hl_codec_encode as source/test_encoder.c does) and only these are kept:
  frame_md5[i]   MD5 of frame i's Annex-B output (header bytes when
                 signalled, 00 00 01, slice NAL) -- EncodeResult.annexb()
  recon_md5[i]   MD5 of frame i's reconstructed (deblocked) picture
  frame_bytes[i] size of frame i's output

Workloads (BENCH_WORKLOADS):
  bench_1088p_s<seed>  bench.py's stream: 1920x1088, QP28, ME 16, deblocking,
                       GOP 30, hartallo_amd.synth.clip(1920, 1088, 150, seed)
                       for seeds 11..18 (bench.py rank r uses seed 11 + r)
  c2_720p_s7           BASELINE config 2 as the reference expresses it
                       (SURVEY §8(d) c2): 1280x720 IPPP GOP 30, QP28, ME 16,
                       31 frames (across the second IDR), seed 7

Run in the build container (needs oracle/_ref/ref_enc):
  python tests/golden/make_bench_golden.py [name ...]     (default: all, in parallel)
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from hartallo_amd import synth  # noqa: E402

REF_ENC = os.path.join(ROOT, "oracle", "_ref", "ref_enc")
OUT = os.path.join(HERE, "bench_golden.json")
BENCH_FRAMES = 150  # bench.py BENCH_CLIP_FRAMES

# name: (W, H, frames, qp, me_range, deblock, gop, seed)
BENCH_WORKLOADS = {f"bench_1088p_s{s}": (1920, 1088, BENCH_FRAMES, 28, 16, 1, 30, s) for s in range(11, 19)}
BENCH_WORKLOADS["c2_720p_s7"] = (1280, 720, 31, 28, 16, 1, 30, 7)


def encode(name):
    w, h, n, qp, mer, db, gop, seed = BENCH_WORKLOADS[name]
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.yuv")
        synth.clip(w, h, n, seed).tofile(inp)
        pre = os.path.join(td, "o")
        r = subprocess.run([REF_ENC, str(w), str(h), str(n), str(qp), str(mer), str(db), str(gop), "0", inp, pre, "rec"],
                           check=True, capture_output=True, text=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        stream = open(pre + ".264", "rb").read()
        ends = [int(v) for v in open(pre + ".idx").read().split()]
        starts = [0] + ends[:-1]
        fs = w * h * 3 // 2
        recon_md5 = []
        with open(pre + ".rec.yuv", "rb") as f:
            for _ in range(n):
                recon_md5.append(hashlib.md5(f.read(fs)).hexdigest())
    return name, {
        "width": w, "height": h, "frames": n, "qp": qp, "me_range": mer, "deblock": db, "gop": gop, "seed": seed,
        "synth": f"hartallo_amd.synth.clip({w}, {h}, {n}, {seed})",
        "stream_md5": hashlib.md5(stream).hexdigest(),
        "frame_md5": [hashlib.md5(stream[a:b]).hexdigest() for a, b in zip(starts, ends)],
        "frame_bytes": [b - a for a, b in zip(starts, ends)],
        "recon_md5": recon_md5,
        "reference_seconds": info["seconds"],
    }


def main():
    if not os.path.exists(REF_ENC):
        sys.exit(f"{REF_ENC} missing: run `make -C oracle ref` where /root/reference exists")
    names = sys.argv[1:] or list(BENCH_WORKLOADS)
    table = json.load(open(OUT)) if os.path.exists(OUT) else {}
    with ThreadPoolExecutor(max_workers=min(8, len(names))) as ex:
        for name, entry in ex.map(encode, names):
            table[name] = entry
            print(f"{name}: {len(entry['frame_md5'])} frames, {sum(entry['frame_bytes'])} bytes, {entry['reference_seconds']:.0f} s", flush=True)
            with open(OUT, "w") as f:
                json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
