"""Parity of frame-pipelined runs (hl_amd_encode_batch, hl_pipeline.h).

A batch must produce exactly the bitstream and reconstruction of the same
frames encoded one call at a time -- which test_gpu_parity.py pins to the
reference -- and of the golden streams the reference itself produced.  The
pipeline geometry is varied so that the cross-picture waits are exercised
with few workgroups (down to the single one that claims tasks in run order),
narrow and wide windows and no guaranteed reach (every partition search then
waits on the reference picture's progress).
Tolerance: none.
"""
import json
import os

import numpy as np
import pytest
import torch

from hartallo_amd import Encoder, synth
from hl_testlib import GOLDEN, GOLDEN_CONFIGS, GOLDEN_ET_CONFIGS, OracleEncoder, first_diff, first_record_diff, golden_input, md5

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


def _device_frames(clip, w, h):
    dev = torch.from_numpy(np.ascontiguousarray(clip)).cuda()
    torch.cuda.synchronize()
    n = w * h
    return dev, [(dev[i].data_ptr(), dev[i].data_ptr() + n, dev[i].data_ptr() + n + n // 4) for i in range(len(clip))]


def _batch(w, h, qp, mer, db, gop, clip, geometry=None, split=None, records=None, et=0):
    enc = Encoder(w, h, qp, mer, db, gop, et)
    if geometry:
        enc.set_pipeline(*geometry)
    dev, ptrs = _device_frames(clip, w, h)
    out, bounds = [], split or [len(ptrs)]
    i = 0
    for n in bounds:
        out += enc.encode_batch_device(ptrs[i:i + n])
        if records is not None:
            records += [enc.debug_records(k) for k in range(n)]
        i += n
    rec = np.concatenate(enc.recon())
    enc.close()
    return [r.annexb() for r in out], rec


def _single(w, h, qp, mer, db, gop, clip, records=None, et=0):
    enc = Encoder(w, h, qp, mer, db, gop, et)
    dev, ptrs = _device_frames(clip, w, h)
    out = []
    for p in ptrs:
        out.append(enc.encode_device(*p).annexb())
        if records is not None:
            records.append(enc.debug_records(0))
    rec = np.concatenate(enc.recon())
    enc.close()
    return out, rec


def _diagnose(w, h, qp, mer, db, gop, clip, geometry=None, split=None, et=0):
    """On a mismatch: the first (picture, MB, field) where the pipelined
    run's decisions differ from one-call-per-picture encoding."""
    ra, rb = [], []
    _single(w, h, qp, mer, db, gop, clip, ra, et)
    _batch(w, h, qp, mer, db, gop, clip, geometry, split, rb, et)
    return first_record_diff(ra, rb, w // 16)


BATCH_GOLDEN = [c for c in GOLDEN_CONFIGS + GOLDEN_ET_CONFIGS if c[3] >= 3]


@pytest.mark.parametrize("cfg", BATCH_GOLDEN, ids=[c[0] for c in BATCH_GOLDEN])
def test_batch_golden_streams(gpu, cfg):
    name, w, h, n, qp, mer, db, gop, seed = cfg
    et = GOLD[name].get("early_term", 0)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    clip = golden_input(cfg)
    out, rec = _batch(w, h, qp, mer, db, gop, clip, et=et)
    got = b"".join(out)
    if got != ref:
        pytest.fail(f"{name}: first differing byte {first_diff(got, ref)}; {_diagnose(w, h, qp, mer, db, gop, clip, et=et)}")
    assert md5(rec) == GOLD[name]["recon_md5"][n - 1]


@pytest.mark.parametrize("w,h", [(16, 16), (32, 16), (48, 16)], ids=["16x16", "32x16", "48x16"])
def test_batch_tiny_pictures_long_run(gpu, w, h):
    """Pictures of fewer macroblocks than ready sub-queues in a run of more
    than 64 pictures: every sub-queue head / tail of every picture slot is
    initialised (k_pipe_init), and the 130 pictures (two runs: 128 + 2,
    across GOPs of 40) equal the reference-pinned oracle's."""
    n = 130
    clip = synth.clip(w, h, n, 71 + w)
    got, rec = _batch(w, h, 28, 8, 1, 40, clip)
    o = OracleEncoder(w, h, 28, 8, 1, 40)
    for f in range(n):
        want = o.encode(clip[f])
        assert got[f] == want, f"{w}x{h} picture {f}: first differing byte {first_diff(got[f], want)}"
    assert np.array_equal(rec, o.recon())


@pytest.mark.parametrize("geometry", [(240, 2, 4), (8, 0, 2), (5, 1, 3), (2, 0, 6), (16, 2, 1), (1, 0, 8), (3, 0, 64)], ids=lambda g: "x".join(map(str, g)))
def test_batch_equals_single_calls(gpu, geometry):
    w, h, n = 320, 240, 9
    clip = synth.clip(w, h, n, 31)
    a, ra = _single(w, h, 26, 16, 1, 30, clip)
    b, rb = _batch(w, h, 26, 16, 1, 30, clip, geometry, split=[1, 5, 3])
    for f in range(n):
        if a[f] != b[f]:
            pytest.fail(f"frame {f}: first differing byte {first_diff(a[f], b[f])}; "
                        f"{_diagnose(w, h, 26, 16, 1, 30, clip, geometry, [1, 5, 3])}")
    assert np.array_equal(ra, rb)


def test_batch_gop_boundaries(gpu):
    # IDR pictures inside the batch split it into pipelined P runs
    w, h, n = 176, 144, 11
    clip = synth.clip(w, h, n, 32)
    a, ra = _single(w, h, 30, 8, 1, 4, clip)
    b, rb = _batch(w, h, 30, 8, 1, 4, clip, (6, 0, 2))
    assert a == b
    assert np.array_equal(ra, rb)


def test_batch_720p_vs_oracle(gpu):
    w, h, n = 1280, 720, 4
    clip = synth.clip(w, h, n, 7)
    out, rec = _batch(w, h, 28, 16, 1, 30, clip)
    o = OracleEncoder(w, h, 28, 16, 1, 30)
    for f in range(n):
        ob = o.encode(clip[f])
        assert out[f] == ob, f"frame {f}: first differing byte {first_diff(out[f], ob)}"
    assert np.array_equal(rec, o.recon())


def test_batch_1088p_equals_single_calls(gpu):
    # the bench workload: 1920x1088, QP28, ME 16, deblocking
    w, h, n = 1920, 1088, 5
    clip = synth.clip(w, h, n, 11)
    a, ra = _single(w, h, 28, 16, 1, 30, clip)
    b, rb = _batch(w, h, 28, 16, 1, 30, clip)
    for f in range(n):
        if a[f] != b[f]:
            pytest.fail(f"frame {f}: first differing byte {first_diff(a[f], b[f])}; {_diagnose(w, h, 28, 16, 1, 30, clip)}")
    assert np.array_equal(ra, rb)


def test_batch_1088p_spans_gops(gpu):
    # runs span GOPs: IDR pictures inside one pipelined launch, whose row-start
    # rdo.Single_ctr reads are resolved exactly in-kernel (no host re-run)
    w, h, n = 1920, 1088, 7
    clip = synth.clip(w, h, n, 13)
    a, ra = _single(w, h, 28, 16, 1, 3, clip)
    enc = Encoder(w, h, 28, 16, 1, 3)
    dev, ptrs = _device_frames(clip, w, h)
    b = [r.annexb() for r in enc.encode_batch_device(ptrs)]
    reruns, launches = enc.last_reruns(), enc.last_mb_launches()
    rb = np.concatenate(enc.recon())
    enc.close()
    for f in range(n):
        if a[f] != b[f]:
            pytest.fail(f"frame {f}: first differing byte {first_diff(a[f], b[f])}; {_diagnose(w, h, 28, 16, 1, 3, clip)}")
    assert np.array_equal(ra, rb)
    assert launches == 1 and reruns == 0, (launches, reruns)


@pytest.mark.parametrize("geometry", [(1, 0, 8), (2, 2, 4)], ids=lambda g: "x".join(map(str, g)))
def test_batch_idr_in_run_few_workgroups(gpu, geometry):
    # 1088p, GOP 3, 4 pictures in one launch (I P P I): the I pictures' exact
    # row-start rdo.Single_ctr walks (resolve_chain) wait mid-task on the end
    # of an earlier row.  With one or two workgroups that row must be held by
    # a running workgroup (claim_next), or the run stalls until a bounded wait
    # gives up and the host re-encodes it.
    w, h, n = 1920, 1088, 4
    clip = synth.clip(w, h, n, 13)
    a, ra = _single(w, h, 28, 16, 1, 3, clip)
    enc = Encoder(w, h, 28, 16, 1, 3)
    enc.set_pipeline(*geometry)
    dev, ptrs = _device_frames(clip, w, h)
    b = [r.annexb() for r in enc.encode_batch_device(ptrs)]
    reruns, launches, walks = enc.last_reruns(), enc.last_mb_launches(), enc.last_chain_walks()
    rb = np.concatenate(enc.recon())
    enc.close()
    assert a == b
    assert np.array_equal(ra, rb)
    assert launches == 1 and reruns == 0, (launches, reruns)
    assert walks > 0  # the case this test is about did occur
