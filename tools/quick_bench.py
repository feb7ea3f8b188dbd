"""Quick timing of a library build variant on the bench workload.

  python tools/quick_bench.py LIB [frames]

Encodes `frames` frames of the 1920x1088 bench clip (inputs in HBM) and
prints per-frame wall and MB-wavefront time.  Development tool only.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hartallo_amd import _lib, synth  # noqa: E402


def main():
    lib = os.path.abspath(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    _lib.load_library(lib)
    import torch

    W, H = 1920, 1088
    clip = synth.clip(W, H, n, 11)
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny, nc = W * H, W * H // 4
    enc = _lib.Encoder(W, H, 28, 16, 1, 30)
    enc.set_timing(True)
    tot = 0.0
    for f in range(n):
        p = dev[f].data_ptr()
        t = time.perf_counter()
        enc.encode_device(p, p + ny, p + ny + nc, collect=False)
        dt = time.perf_counter() - t
        ms = enc.timing_ms()
        if f:
            tot += dt
        print(f"{os.path.basename(os.path.dirname(lib))} frame {f}: wall {dt * 1e3:.1f} ms  mb {ms[1]:.1f} ms  deblock {ms[2]:.2f} ms", flush=True)
    print(f"{lib}: mean P-frame {tot / max(1, n - 1) * 1e3:.1f} ms", flush=True)
    enc.close()


if __name__ == "__main__":
    main()
