"""Per-phase cycle breakdown of the macroblock kernel (profiling build,
`make profile`): lane 0 of every workgroup accumulates clock64() deltas.

  python tools/phase_profile.py [frames]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hartallo_amd  # noqa: E402
from hartallo_amd import _lib, synth  # noqa: E402

PHASES = ["eval:block", "eval:nC", "eval:reduce", "search_partition", "mvp", "guess_intra(P)", "mb_begin", "mb_end", "whole MB",
          "reach_wait", "intra:i16", "intra:i4", "step:slots+loads", "step:fwd+quant", "step:idct+cavlc", "step:-", "step:candidates",
          "step:selection", "sel:resolve", "cand:generate"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    _lib.load_library(os.environ.get("HL_LIB") or os.path.join(ROOT, "build", "prof", "hartallo_amd", "libhartallo_amd.so"))
    W, H = 1920, 1088
    clip = synth.clip(W, H, n, 11)
    enc = hartallo_amd.Encoder(W, H, 28, 16, 1, 30)
    enc.set_timing(True)
    for f in range(n):
        t = time.perf_counter()
        y = clip[f]
        enc.encode(y[:W * H], y[W * H:W * H * 5 // 4], y[W * H * 5 // 4:])
        dt = time.perf_counter() - t
        ms = enc.timing_ms()
        print(f"frame {f}: wall {dt * 1e3:.1f} ms  planes {ms[0]:.2f}  mb {ms[1]:.1f}  deblock {ms[2]:.2f}  device {ms[3]:.1f} ms  reruns {enc.last_reruns()}")
        nmb = (W // 16) * (H // 16)
        cnt = enc.profile_counters(64 + nmb)
        mbc = np.array(cnt[64:64 + nmb], dtype=np.float64).reshape(H // 16, W // 16)
        # launch-per-diagonal time (sum of per-diagonal maxima) vs the dataflow
        # critical path (MB (x, y) after (x-1, y) and (x+1, y-1))
        mbh, mbw = mbc.shape
        diag_max = sum(max((mbc[y, d - 2 * y] for y in range(mbh) if 0 <= d - 2 * y < mbw), default=0.0) for d in range(mbw + 2 * mbh))
        fin = np.zeros_like(mbc)
        for y in range(mbh):
            for x in range(mbw):
                dep = max(fin[y, x - 1] if x else 0.0, fin[y - 1, x + 1] if y and x + 1 < mbw else (fin[y - 1, x] if y else 0.0))
                fin[y, x] = dep + mbc[y, x]
        print(f"   MB cycles: mean {mbc.mean():.0f}  max {mbc.max():.0f}  sum-of-diagonal-max {diag_max / 1e6:.1f} M  dataflow critical path {fin.max() / 1e6:.1f} M")
        for i, name in enumerate(PHASES):
            cyc, calls = cnt[2 * i], cnt[2 * i + 1]
            if calls:
                print(f"   {name:18s} calls/MB {calls / nmb:8.1f}  cycles/call {cyc / calls:10.0f}  kcycles/MB {cyc / nmb / 1e3:9.1f}")


if __name__ == "__main__":
    main()
