"""Development probe (GPU): where the time of each per-picture call goes on
the bench stream -- wall time, kernel time (HIP events), how the call ran
(runs / per-picture fallbacks / chain walks / re-runs) and the helpers'
counts -- picture by picture, and each picture's MD5 against the reference
encoder's (tests/golden/bench_golden.json).

  python tools/per_call_probe.py [frames] [name]
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hartallo_amd import _lib, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    name = sys.argv[2] if len(sys.argv) > 2 else "bench_1088p_s11"
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_golden.json")))[name]
    w, h = g["width"], g["height"]
    clip = synth.clip(w, h, g["frames"], g["seed"])[:n]
    enc = _lib.Encoder(w, h, qp=g["qp"], me_range=g["me_range"], deblock=g["deblock"], gop_size=g["gop"])
    enc.set_timing(True)
    ny, nc = w * h, w * h // 4
    for i in range(n):
        f = clip[i].reshape(-1)
        t0 = time.perf_counter()
        r = enc.encode(f[:ny], f[ny:ny + nc], f[ny + nc:])
        ms = 1e3 * (time.perf_counter() - t0)
        out = r.annexb()
        print(json.dumps({"frame": i, "wall_ms": round(ms, 2), "timing_ms": [round(x, 2) for x in enc.timing_ms()],
                          "md5_ok": hashlib.md5(out).hexdigest() == g["frame_md5"][i], "reruns": enc.last_reruns(),
                          "batch": enc.last_batch_stats(), "helpers": enc.last_helper_stats()}), flush=True)


if __name__ == "__main__":
    main()
