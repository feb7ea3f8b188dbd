"""Parity of the gfx950 encode path (libhartallo_amd.so, through the C ABI)
against the reference.

* golden: every configuration of tests/golden/ (streams produced by the
  reference encoder itself, oracle/_ref/ref_enc) must be reproduced byte for
  byte, and the reconstructed pictures must match the reference's MD5s;
* oracle: larger seeded clips (720p, 1920x1088) must match the bit-exact CPU
  restatement (oracle/hl_oracle.c) byte for byte, recon included;
* full-size properties at the bench configuration.
Tolerance: none -- the path is integer (double only inside RDO costs, which
are compared by decision, i.e. by the bitstream).
"""
import json
import os

import numpy as np
import pytest

from hl_testlib import GOLDEN, GOLDEN_CONFIGS, GOLDEN_ET_CONFIGS, GOLDEN_MRF_CONFIGS, GOLDEN_RC_CONFIGS, GpuEncoder, OracleEncoder, first_diff, golden_input, md5

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


ALL = GOLDEN_CONFIGS + GOLDEN_ET_CONFIGS


@pytest.mark.parametrize("cfg", ALL, ids=[c[0] for c in ALL])
def test_golden_streams(gpu, cfg):
    name, w, h, n, qp, mer, db, gop, seed = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = GpuEncoder(w, h, qp, mer, db, gop, GOLD[name].get("early_term", 0))
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f} differs"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"


@pytest.mark.parametrize("cfg", GOLDEN_MRF_CONFIGS, ids=[c[0] for c in GOLDEN_MRF_CONFIGS])
def test_max_ref_frame_golden_streams(gpu, cfg):
    """hl_codec_t.max_ref_frame > 1 (hl_amd_set_max_ref_frame): per call and
    as one batch (the pipelined runs), both equal to the reference's stream."""
    import torch

    from hartallo_amd import Encoder

    name, w, h, n, qp, mer, db, gop, seed, mrf = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = GpuEncoder(w, h, qp, mer, db, gop, 0, mrf)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f} differs"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"
    dev = torch.from_numpy(np.ascontiguousarray(clip)).cuda()
    torch.cuda.synchronize()
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + w * h, dev[i].data_ptr() + w * h * 5 // 4) for i in range(n)]
    b = Encoder(w, h, qp, mer, db, gop)
    b.set_max_ref_frame(mrf)
    got = b"".join(r.annexb() for r in b.encode_batch_device(ptrs))
    with pytest.raises(Exception):
        b.set_max_ref_frame(1)  # after the first frame: the headers are out (INVALID_STATE)
    b.close()
    assert got == ref, f"{name} (batch): first differing byte {first_diff(got, ref)}"


@pytest.mark.parametrize("cfg", GOLDEN_RC_CONFIGS, ids=[c[0] for c in GOLDEN_RC_CONFIGS])
def test_rate_control_golden_streams(gpu, cfg):
    """rc_bitrate > 0 (hl_codec_264.c:719-742): per-picture QPs from the rate
    controller, streams and recon identical to the reference's."""
    name, w, h, n, qp, mer, db, gop, seed, br, bu, qmin, qmax = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    g = GOLD[name]
    enc = GpuEncoder(w, h, qp, mer, db, gop)
    enc.set_rate_control(br, g["fps_num"], g["fps_den"], bu, qmin, qmax)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert enc.last_qp() == g["slice_qp"][f], f"{name}: QP of frame {f}"
        assert md5(enc.recon()) == g["recon_md5"][f], f"{name}: recon of frame {f} differs"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"


def test_rate_control_batch_equals_calls(gpu):
    """Under rate control hl_amd_encode_batch codes picture by picture and
    returns the same stream as one call per frame."""
    import torch

    from hartallo_amd import Encoder

    cfg = GOLDEN_RC_CONFIGS[0]
    name, w, h, n, qp, mer, db, gop, seed, br, bu, qmin, qmax = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    dev = torch.from_numpy(clip).cuda()
    ny = w * h
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(n)]
    enc = Encoder(w, h, qp, mer, db, gop)
    enc.set_rate_control(br, 1, 15, bu, qmin, qmax)
    out = b"".join(r.annexb() for r in enc.encode_batch_device(ptrs))
    enc.close()
    assert out == ref, f"first differing byte {first_diff(out, ref)}"


def _vs_oracle(w, h, n, qp, mer, db, gop, seed):
    clip = np.stack([np.concatenate([y.ravel(), u.ravel(), v.ravel()]) for y, u, v in __import__("hartallo_amd.synth", fromlist=["frames"]).frames(w, h, n, seed)])
    g = GpuEncoder(w, h, qp, mer, db, gop)
    o = OracleEncoder(w, h, qp, mer, db, gop)
    for f in range(n):
        a, b = g.encode(clip[f]), o.encode(clip[f])
        assert a == b, f"frame {f}: first differing byte {first_diff(a, b)}"
        assert np.array_equal(g.recon(), o.recon()), f"frame {f}: recon differs"


def test_720p_ipp_vs_oracle(gpu):
    _vs_oracle(1280, 720, 3, 28, 16, 1, 30, 7)


def test_1088p_ip_vs_oracle(gpu):
    # the bench workload (1920x1088 IPPP, QP28, ME 16, deblock) for 2 frames
    _vs_oracle(1920, 1088, 2, 28, 16, 1, 30, 11)


def test_gop2_short_frames_vs_oracle(gpu):
    # I P I P ... with state leaking across GOPs (per-address MB objects)
    _vs_oracle(320, 240, 5, 26, 8, 1, 2, 21)


def test_fails_where_reference_fails(gpu):
    """QP 8: the reference's lambda is negative (slice.c:1766 with x86's
    shift-count masking, hl_prims.h rdo_lambda) and its first P picture's
    slice outgrows the slice buffer: HL_ERROR_TOOSHORT.  The GPU encoder
    codes the I picture byte for byte and refuses the P picture with the same
    error, per call and batched."""
    from hartallo_amd import HlAmdError

    from hl_testlib import check_reference_failure

    g = GOLD["fail_qcif_qp8_neg_lambda"]

    def enc_ok(e, frame):
        try:
            return e.encode(frame)
        except HlAmdError as x:
            assert x.code == g["fail_error"], f"refused with {x.code}, the reference with {g['fail_error']}"
            return None

    check_reference_failure("fail_qcif_qp8_neg_lambda", lambda c: GpuEncoder(c[1], c[2], c[4], c[5], c[6], c[7]), enc_ok, GOLD)


def test_rejects_bad_format(gpu):
    from hartallo_amd import Encoder, HlAmdError

    with pytest.raises(HlAmdError) as e:
        Encoder(1920, 1080)
    assert e.value.code == 4  # HL_ERROR_INVALID_FORMAT, hl_codec_264.c:437-438
    with pytest.raises(HlAmdError) as e:
        Encoder(32, 16, me_early_term=1)  # early termination reads one sample around the MB quadrants
    assert e.value.code == 4


def test_early_term_720p_vs_oracle(gpu):
    # me_early_term_flag = 1 is the hl_codec_create default (hl_types.h:67)
    w, h, n = 1280, 720, 3
    clip = __import__("hartallo_amd.synth", fromlist=["clip"]).clip(w, h, n, 7)
    g = GpuEncoder(w, h, 28, 16, 1, 30, 1)
    o = OracleEncoder(w, h, 28, 16, 1, 30, 1)
    for f in range(n):
        a, b = g.encode(clip[f]), o.encode(clip[f])
        assert a == b, f"frame {f}: first differing byte {first_diff(a, b)}"
        assert np.array_equal(g.recon(), o.recon()), f"frame {f}: recon differs"
