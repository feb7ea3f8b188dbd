"""Where the time of one P picture goes along its critical path (profiling
build, build/prof): the picture is encoded alone (one call, a pipelined run
of one) and every MB's task records, on the wall clock, when its workgroup
took it, when its decision ended and when its in-picture successors were
released.  From those the tool walks the critical path back from the last MB
(each step to the dependency -- (x-1, y) or (x+1, y-1) -- released last) and
splits every step into: the hand-over (the dependency's release until the
task was taken), the task start and decision, and the release after it.

  python tools/critical_path.py [pictures-before]      (development tool)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hartallo_amd import _lib  # noqa: E402

_lib.load_library(os.environ.get("HL_LIB") or os.path.join(ROOT, "build", "prof", "hartallo_amd", "libhartallo_amd.so"))
from hartallo_amd import Encoder, synth  # noqa: E402

TICK_US = 0.01  # s_memrealtime: 100 MHz


def main():
    before = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    W, H = 1920, 1088
    mbw, mbh = W // 16, H // 16
    nmb = mbw * mbh
    clip = synth.clip(W, H, before + 1, 11)
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny = W * H
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(before + 1)]
    enc = Encoder(W, H, 28, 16, 1, 30)
    if os.environ.get("HL_PROF_HELPERS") == "0":
        enc.set_intra_helpers(False)
    for i in range(before):
        enc.encode_device(*ptrs[i], collect=False)
    enc.profile_counters(64)
    torch.cuda.synchronize()
    enc.encode_device(*ptrs[before], collect=False)
    torch.cuda.synchronize()
    cnt = np.array(enc.profile_counters(64 + 4 * nmb), dtype=np.float64)
    tl = cnt[64 + nmb:64 + 4 * nmb].reshape(mbh, mbw, 3)
    t0 = tl[..., 0][tl[..., 0] > 0].min()
    tl = (tl - t0) * TICK_US
    start, end, rel = tl[..., 0], tl[..., 1], tl[..., 2]
    # walk back from the last MB
    x, y = mbw - 1, mbh - 1
    steps = []
    while True:
        deps = []
        if x > 0:
            deps.append((x - 1, y))
        if y > 0:
            deps.append((min(x + 1, mbw - 1), y - 1))
        if not deps:
            steps.append((x, y, 0.0, start[y, x], end[y, x] - start[y, x], rel[y, x] - end[y, x]))
            break
        dx, dy = max(deps, key=lambda d: rel[d[1], d[0]])
        steps.append((x, y, rel[dy, dx], start[y, x] - rel[dy, dx], end[y, x] - start[y, x], rel[y, x] - end[y, x]))
        x, y = dx, dy
    steps.reverse()
    hand = np.array([s[3] for s in steps[1:]])
    dec = np.array([s[4] for s in steps])
    rls = np.array([s[5] for s in steps])
    total = rel[mbh - 1, mbw - 1]
    print(f"picture {before} (P) alone: last MB released at {total / 1e3:.2f} ms; critical path {len(steps)} MBs")
    print(f"   per step: hand-over {hand.mean():.1f} us (median {np.median(hand):.1f}, max {hand.max():.1f}), "
          f"task start + decision {dec.mean():.1f} us (median {np.median(dec):.1f}), release {rls.mean():.1f} us")
    print(f"   sums: hand-over {hand.sum() / 1e3:.2f} ms, decisions {dec.sum() / 1e3:.2f} ms, releases {rls.sum() / 1e3:.2f} ms")
    print(f"   all MBs: decision mean {(end - start).mean():.1f} us, release mean {(rel - end).mean():.1f} us")
    enc.close()


if __name__ == "__main__":
    main()
