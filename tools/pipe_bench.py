"""Timing of pipelined runs on the bench workload for several geometries.

  python tools/pipe_bench.py [frames] [workgroups,R,window ...]

Development tool: 1920x1088 QP28 ME16 deblock; two warm-up pictures (I, P)
one call at a time, then `frames` P pictures in one hl_amd_encode_batch.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hartallo_amd import _lib  # noqa: E402

if os.environ.get("HL_LIB"):  # development: time another build of the library
    _lib.load_library(os.path.abspath(os.environ["HL_LIB"]))
from hartallo_amd import Encoder, synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    geos = [tuple(map(int, g.split(","))) for g in sys.argv[2:]] or [(0, 2, 64)]
    W, H = 1920, 1088
    clip = synth.clip(W, H, n + 2, 11)
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny, nc = W * H, W * H // 4
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + nc) for i in range(n + 2)]
    for g in geos:
        enc = Encoder(W, H, 28, 16, 1, 30)
        enc.set_pipeline(*g)
        enc.set_timing(True)
        for i in range(2):
            enc.encode_device(*ptrs[i], collect=False)
        t = time.perf_counter()
        nbytes = enc.encode_batch_device(ptrs[2:], collect=False)
        dt = time.perf_counter() - t
        ms = enc.timing_ms()
        print(f"wg,R,window={g}: {n} P pictures in {dt * 1e3:.1f} ms = {n / dt:.2f} fps (kernel {ms[1]:.1f} ms, reruns {enc.last_reruns()}, {nbytes} bytes)",
              flush=True)
        enc.close()


if __name__ == "__main__":
    main()
