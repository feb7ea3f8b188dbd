"""Several streams per GPU in one process (hl_amd_encode_streams): every
stream's pictures in shared pipelined runs.  Each stream is one encoder with
its own seed; every frame of every stream must match the reference
encoder's per-frame MD5s for that seed (tests/golden/bench_golden.json,
1920x1088, QP28, ME16, deblocking, GOP 30), exactly as if that encoder had
coded its stream alone (the reference serves N streams as N hl_codec_t
instances, hl_codec.c:24-150)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from hartallo_amd import Encoder, HlAmdError, synth
from hl_testlib import GOLDEN

pytestmark = pytest.mark.gpu

BENCH = json.load(open(os.path.join(GOLDEN, "bench_golden.json")))


def _streams(seeds, n):
    devs, ptrs = [], []
    for sd in seeds:
        g = BENCH[f"bench_1088p_s{sd}"]
        w, h = g["width"], g["height"]
        dev = torch.from_numpy(np.ascontiguousarray(synth.clip(w, h, g["frames"], sd)[:n])).cuda()
        devs.append(dev)
        ny = w * h
        ptrs.append([(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(n)])
    torch.cuda.synchronize()
    return devs, ptrs


@pytest.mark.parametrize("count", [2, 4])
def test_streams_share_one_launch(gpu, count):
    seeds = list(range(11, 11 + count))
    warm, steps = 5, 20  # the driver's shape: a warm-up call, then 20 frames per stream
    devs, ptrs = _streams(seeds, warm + steps)
    g = BENCH["bench_1088p_s11"]
    encs = [Encoder(g["width"], g["height"], g["qp"], g["me_range"], g["deblock"], g["gop"]) for _ in seeds]
    outs = [[] for _ in seeds]
    for lo, hi in ((0, warm), (warm, warm + steps)):
        res = Encoder.encode_streams_device(encs, [p[lo:hi] for p in ptrs])
        for si, rs in enumerate(res):
            outs[si] += [r.annexb() for r in rs]
        for e in encs:  # one clean shared launch, no picture on the per-picture path
            st = e.last_batch_stats()
            assert st["runs"] == 1 and st["per_picture"] == 0 and st["fallbacks"] == 0 and st["waits_gave_up"] == 0, st
            assert e.last_mb_launches() == 1
    for si, sd in enumerate(seeds):
        gold = BENCH[f"bench_1088p_s{sd}"]["frame_md5"]
        for f, o in enumerate(outs[si]):
            assert hashlib.md5(o).hexdigest() == gold[f], f"stream seed {sd} frame {f} differs from the reference"
    for e in encs:
        e.close()


def test_streams_reject_mismatched_encoders(gpu):
    g = BENCH["bench_1088p_s11"]
    a = Encoder(g["width"], g["height"], 28, 16, 1, 30)
    b = Encoder(1280, 720, 28, 16, 1, 30)
    devs, ptrs = _streams([11], 1)
    try:
        with pytest.raises(HlAmdError):  # different picture sizes
            Encoder.encode_streams_device([a, b], [ptrs[0], ptrs[0]])
        with pytest.raises(HlAmdError):  # the same encoder twice
            Encoder.encode_streams_device([a, a], [ptrs[0], ptrs[0]])
    finally:
        a.close()
        b.close()
