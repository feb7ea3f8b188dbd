"""Per-phase cycle breakdown of the macroblock kernel (profiling build,
`make profile`): lane 0 of every workgroup accumulates clock64() deltas.

  python tools/phase_profile.py [frames]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hartallo_amd  # noqa: E402
from hartallo_amd import _lib, synth  # noqa: E402

PHASES = ["eval:block", "eval:nC", "eval:reduce", "search_partition", "mvp", "guess_intra(P)", "mb_begin", "mb_end", "whole MB",
          "-", "intra:i16", "intra:i4"]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    _lib.load_library(os.path.join(ROOT, "build", "prof", "hartallo_amd", "libhartallo_amd.so"))
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
        cnt = enc.profile_counters(2 * len(PHASES))
        print(f"frame {f}: wall {dt * 1e3:.1f} ms  planes {ms[0]:.2f}  mb {ms[1]:.1f}  deblock {ms[2]:.2f}  device {ms[3]:.1f} ms  reruns {enc.last_reruns()}")
        nmb = (W // 16) * (H // 16)
        for i, name in enumerate(PHASES):
            cyc, calls = cnt[2 * i], cnt[2 * i + 1]
            if calls:
                print(f"   {name:18s} calls/MB {calls / nmb:8.1f}  cycles/call {cyc / calls:10.0f}  kcycles/MB {cyc / nmb / 1e3:9.1f}")


if __name__ == "__main__":
    main()
