"""Parity at the BASELINE sizes against the reference encoder itself.

tests/golden/bench_golden.json holds, per frame, the MD5 of the reference
encoder's Annex-B output and of its reconstructed picture for
  * bench.py's stream (1920x1088, QP28, ME 16, deblocking, GOP 30,
    synth.clip(1920, 1088, 150, 11)), and
  * BASELINE config 2 as the reference expresses it (1280x720 IPPP GOP 30,
    QP28, ME 16, 31 frames across the second IDR),
produced by oracle/_ref/ref_enc (tests/golden/make_bench_golden.py).  The
pipelined path (one launch spanning GOPs), the way bench.py and the driver
call it, and the per-picture path must reproduce them.  Tolerance: none.
"""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from hartallo_amd import Encoder, synth
from hl_testlib import GOLDEN

pytestmark = pytest.mark.gpu

BENCH = json.load(open(os.path.join(GOLDEN, "bench_golden.json")))
_CLIPS = {}


def _clip(name):
    if name not in _CLIPS:
        g = BENCH[name]
        _CLIPS[name] = synth.clip(g["width"], g["height"], g["frames"], g["seed"])
    return _CLIPS[name]


def _ptrs(dev, w, h):
    n = w * h
    return [(dev[i].data_ptr(), dev[i].data_ptr() + n, dev[i].data_ptr() + n + n // 4) for i in range(dev.shape[0])]


def _md5(b):
    return hashlib.md5(bytes(b)).hexdigest()


def _check(name, first, outs, recons):
    g = BENCH[name]
    for i, o in enumerate(outs):
        f = first + i
        assert _md5(o) == g["frame_md5"][f], f"{name} frame {f}: output differs from the reference ({len(o)} vs {g['frame_bytes'][f]} bytes)"
    for i, r in enumerate(recons):
        if r is not None:
            assert _md5(r) == g["recon_md5"][first + i], f"{name} frame {first + i}: reconstruction differs from the reference"


def _check_clean_runs(enc, m):
    """The call ran as pipelined runs of up to 128 pictures, with no fallback
    to the per-picture path and no bounded wait that gave up (a silent
    fallback would still produce the right bytes)."""
    st = enc.last_batch_stats()
    assert st == {"runs": (m + 127) // 128, "per_picture": 0, "fallbacks": 0, "waits_gave_up": 0, "chain_walks": st["chain_walks"]}, st
    assert enc.last_mb_launches() == 1 and enc.last_reruns() == 0


def _batch(name, calls, geometry=None):
    """Encodes the stream's first sum(calls) frames with one
    encode_batch_device call per entry of `calls`."""
    g = BENCH[name]
    w, h = g["width"], g["height"]
    n = sum(calls)
    dev = torch.from_numpy(np.ascontiguousarray(_clip(name)[:n])).cuda()
    torch.cuda.synchronize()
    ptrs = _ptrs(dev, w, h)
    enc = Encoder(w, h, g["qp"], g["me_range"], g["deblock"], g["gop"])
    if geometry:
        enc.set_pipeline(*geometry)
    outs, recons, i = [], [], 0
    for m in calls:
        outs += [r.annexb() for r in enc.encode_batch_device(ptrs[i:i + m])]
        _check_clean_runs(enc, m)
        recons += [enc.debug_recon(k) for k in range(m)]
        i += m
    enc.close()
    return outs, recons


def test_bench_stream_driver_calls(gpu):
    # the driver's `bench.py --steps 20 --warmup 5`: a 5-frame warm-up call, then 20 frames
    outs, recons = _batch("bench_1088p_s11", [5, 20])
    _check("bench_1088p_s11", 0, outs, recons)


def test_bench_stream_one_launch_across_gops(gpu):
    # one pipelined launch over 40 pictures: the IDR at frame 30 sits inside the run
    outs, recons = _batch("bench_1088p_s11", [40])
    _check("bench_1088p_s11", 0, outs, recons)


def test_bench_stream_default_run(gpu):
    # bench.py's default: warm-up GOP, then four GOPs in one launch (150 frames)
    outs, recons = _batch("bench_1088p_s11", [30, 120])
    _check("bench_1088p_s11", 0, outs, recons)


def test_bench_stream_other_rank(gpu):
    # rank 3 of a multi-GPU bench encodes seed 14
    outs, recons = _batch("bench_1088p_s14", [5, 20])
    _check("bench_1088p_s14", 0, outs, recons)


def test_bench_stream_per_picture(gpu):
    g = BENCH["bench_1088p_s11"]
    w, h = g["width"], g["height"]
    dev = torch.from_numpy(np.ascontiguousarray(_clip("bench_1088p_s11")[:4])).cuda()
    torch.cuda.synchronize()
    enc = Encoder(w, h, g["qp"], g["me_range"], g["deblock"], g["gop"])
    outs, recons = [], []
    for i, p in enumerate(_ptrs(dev, w, h)):
        outs.append(enc.encode_device(*p).annexb())
        _check_clean_runs(enc, 1)  # one persistent launch per picture
        recons.append(np.concatenate(enc.recon()))
        if i > 0:  # a lone P picture runs its macroblocks' helper tasks
            hs = enc.last_helper_stats()
            assert hs["i4_kept"] > 0 and hs["fam3_kept"] > 0, hs
    enc.close()
    _check("bench_1088p_s11", 0, outs, recons)


def test_bench_stream_lookahead(gpu):
    # host frames through hl_amd_encode with an 8-frame look-ahead: results in
    # order, lookahead - 1 calls late, the rest from flush(); each equals the
    # reference's frame; setting it after the first frame is refused
    g = BENCH["bench_1088p_s11"]
    w, h, n = g["width"], g["height"], 13
    clip = _clip("bench_1088p_s11")[:n]
    enc = Encoder(w, h, g["qp"], g["me_range"], g["deblock"], g["gop"])
    enc.set_lookahead(8)
    outs, got = [], 0
    ny = w * h
    for i in range(n):
        f = clip[i].reshape(-1)
        r = enc.encode(f[:ny], f[ny:ny + ny // 4], f[ny + ny // 4:])
        assert (r.type != 0) == (i >= 7), (i, r.type)
        if r.type:
            outs.append(r.annexb())
    while True:
        r = enc.flush()
        if not r.type:
            break
        outs.append(r.annexb())
    with pytest.raises(Exception):
        enc.set_lookahead(4)
    enc.close()
    assert len(outs) == n
    _check("bench_1088p_s11", 0, outs, [])
    # while frames are queued, device-frame calls are refused (flush first)
    enc = Encoder(w, h, g["qp"], g["me_range"], g["deblock"], g["gop"])
    enc.set_lookahead(4)
    f = clip[0].reshape(-1)
    assert enc.encode(f[:ny], f[ny:ny + ny // 4], f[ny + ny // 4:]).type == 0
    dev = torch.from_numpy(np.ascontiguousarray(clip[:1])).cuda()
    torch.cuda.synchronize()
    with pytest.raises(Exception):
        enc.encode_device(*_ptrs(dev, w, h)[0])
    r = enc.flush()
    assert r.annexb() and not enc.flush().type
    enc.close()
    _check("bench_1088p_s11", 0, [r.annexb()], [])


def test_bench_stream_partitioning_helpers_in_runs(gpu, monkeypatch):
    # the partitioning helpers in a run of one stream (HL_AMD_FAM3=2, read
    # when the encoder opens), for every picture and for the run's edges only
    for edge in ("99,99", "1,2"):
        monkeypatch.setenv("HL_AMD_FAM3", "2")
        monkeypatch.setenv("HL_AMD_F3_EDGE", edge)
        outs, recons = _batch("bench_1088p_s11", [3, 8])
        _check("bench_1088p_s11", 0, outs, recons)


def test_config2_720p_pipelined(gpu):
    outs, recons = _batch("c2_720p_s7", [31])
    _check("c2_720p_s7", 0, outs, recons)


def test_config2_720p_per_picture(gpu):
    g = BENCH["c2_720p_s7"]
    w, h = g["width"], g["height"]
    dev = torch.from_numpy(np.ascontiguousarray(_clip("c2_720p_s7"))).cuda()
    torch.cuda.synchronize()
    enc = Encoder(w, h, g["qp"], g["me_range"], g["deblock"], g["gop"])
    outs, recons = [], []
    for p in _ptrs(dev, w, h):
        outs.append(enc.encode_device(*p).annexb())
        _check_clean_runs(enc, 1)
        recons.append(np.concatenate(enc.recon()))
    enc.close()
    _check("c2_720p_s7", 0, outs, recons)


def test_bench_stream_per_picture_fallback(gpu, monkeypatch):
    # the per-picture wavefront path (what a run falls back to) on the bench stream
    monkeypatch.setenv("HL_AMD_FORCE_FALLBACK", "1")
    g = BENCH["bench_1088p_s11"]
    dev = torch.from_numpy(np.ascontiguousarray(_clip("bench_1088p_s11")[:3])).cuda()
    torch.cuda.synchronize()
    enc = Encoder(g["width"], g["height"], g["qp"], g["me_range"], g["deblock"], g["gop"])
    outs = [r.annexb() for r in enc.encode_batch_device(_ptrs(dev, g["width"], g["height"]))]
    st = enc.last_batch_stats()
    assert st["fallbacks"] == 1 and st["per_picture"] == 3, st
    recons = [enc.debug_recon(k) for k in range(3)]
    enc.close()
    _check("bench_1088p_s11", 0, outs, recons)
