"""The gfx950 kernel logic (hartallo_amd/csrc/hl_mbcore.h, hl_filters.h),
compiled for the host with one lane per workgroup (tests/emu/libhl_emu.so),
together with the product's host bitstream writer must reproduce the
reference's golden streams byte for byte.  This checks the kernel logic and
the writer without a GPU; the GPU itself is checked by test_gpu_parity.py."""
import ctypes
import json
import os

import pytest

from hl_testlib import (EMU_LIB, GOLDEN, GOLDEN_CONFIGS, GOLDEN_ET_CONFIGS, GOLDEN_MRF_CONFIGS, GOLDEN_RC_CONFIGS, EmuEncoder, OracleEncoder, first_diff,
                        golden_input, md5)
from hartallo_amd import synth

GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


ALL = GOLDEN_CONFIGS + GOLDEN_ET_CONFIGS


@pytest.mark.parametrize("cfg", ALL, ids=[c[0] for c in ALL])
def test_kernel_logic_matches_reference(cfg):
    name, w, h, n, qp, mer, db, gop, seed = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = EmuEncoder(w, h, qp, mer, db, gop, GOLD[name].get("early_term", 0))
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"


@pytest.mark.parametrize("cfg", GOLDEN_MRF_CONFIGS, ids=[c[0] for c in GOLDEN_MRF_CONFIGS])
def test_max_ref_frame_matches_reference(cfg):
    """hl_codec_t.max_ref_frame > 1 through the product's writer
    (sps_max_num_ref_frames, hl_writer.cpp)."""
    name, w, h, n, qp, mer, db, gop, seed, mrf = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = EmuEncoder(w, h, qp, mer, db, gop, 0, mrf)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"


@pytest.mark.parametrize("mode", [1, 2], ids=["helpers", "helpers_bad_guess"])
@pytest.mark.parametrize("cfg", ALL, ids=[c[0] for c in ALL])
def test_intra_helpers_match_reference(cfg, mode):
    """Every P macroblock's intra fallback prepared by its intra helper
    (hl_mbcore.h intra_helper, as a pipelined run's helper task runs it) and
    resolved against the live state (i16_light, i4_verify): the same streams.
    mode 2 makes the helpers guess the live TotalCoeffs wrongly, so that
    i4_verify's rejections and the macroblock's own Intra4x4 are exercised."""
    name, w, h, n, qp, mer, db, gop, seed = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = EmuEncoder(w, h, qp, mer, db, gop, GOLD[name].get("early_term", 0))
    enc.lib.emu_set_helper(ctypes.c_void_p(enc.h_), mode)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"
    kept = enc.lib.emu_helper_i4(ctypes.c_void_p(enc.h_), 0)
    rejected = enc.lib.emu_helper_i4(ctypes.c_void_p(enc.h_), 1)
    if any(f % gop for f in range(n)):  # P pictures: every P macroblock with an intra trial used its helper
        assert kept + rejected > 0
    if mode == 1:  # the natural guess: the helper's Intra4x4 is nearly always kept
        assert rejected <= max(8, (kept + rejected) // 20), (kept, rejected)


def test_intra_helpers_bad_guess_rejects():
    """The wrong guess is rejected somewhere in the golden set (the
    rejection path is covered, not only the acceptance)."""
    rej = 0
    for cfg in ALL[:6]:
        name, w, h, n, qp, mer, db, gop, seed = cfg
        clip = golden_input(cfg)
        enc = EmuEncoder(w, h, qp, mer, db, gop, GOLD[name].get("early_term", 0))
        enc.lib.emu_set_helper(ctypes.c_void_p(enc.h_), 2)
        for f in range(n):
            enc.encode(clip[f])
        rej += enc.lib.emu_helper_i4(ctypes.c_void_p(enc.h_), 1)
    assert rej > 0


@pytest.mark.parametrize("cfg", GOLDEN_RC_CONFIGS, ids=[c[0] for c in GOLDEN_RC_CONFIGS])
def test_rate_control_matches_reference(cfg):
    """The product's rate control (hartallo_amd/csrc/hl_rc.cpp) driving the
    kernel logic reproduces the reference's rate-controlled streams: every
    picture's QP (hl_codec_264_rc.c model), stream and recon."""
    name, w, h, n, qp, mer, db, gop, seed, br, bu, qmin, qmax = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    g = GOLD[name]
    enc = EmuEncoder(w, h, qp, mer, db, gop)
    enc.set_rate_control(br, g["fps_num"], g["fps_den"], bu, qmin, qmax)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert enc.last_qp() == g["slice_qp"][f], f"{name}: QP of frame {f}"
        assert md5(enc.recon()) == g["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"


@pytest.mark.parametrize("seed", [31, 32, 33, 34])
def test_kernel_logic_matches_oracle_random_params(seed):
    import numpy as np

    rng = np.random.default_rng(seed)
    w, h = 16 * int(rng.integers(2, 12)), 16 * int(rng.integers(1, 9))
    qp, mer, db, gop = int(rng.integers(0, 52)), int(rng.integers(1, 33)), int(rng.integers(0, 2)), int(rng.integers(1, 6))
    clip = synth.clip(w, h, 5, seed)
    et = int(rng.integers(0, 2)) if w >= 32 and h >= 32 else 0
    a, b = EmuEncoder(w, h, qp, mer, db, gop, et), OracleEncoder(w, h, qp, mer, db, gop, et)
    for f in range(len(clip)):
        x, y = a.encode(clip[f]), b.encode(clip[f])
        assert x == y, f"{w}x{h} qp{qp} me{mer} db{db} gop{gop} frame {f}: byte {first_diff(x, y)}"


def test_level_code_lengths_match_writer_table():
    """The GPU CAVLC bit counter (hl_prims.h level_code_len) and the writer's
    generated level table (cavlc.c:59-103 semantics) agree everywhere."""
    lib = ctypes.CDLL(EMU_LIB)
    for sl in range(7):
        for lc in list(range(0, 5000)) + list(range(5000, 62546, 37)):
            assert lib.emu_level_code_len(sl, lc) == lib.emu_writer_level_bits(sl, lc), (sl, lc)


def test_i4_prediction_table():
    """The GPU's branch-free Intra4x4 prediction (hl_mbcore.h kI4Tab: three
    taps and weights per mode and sample, derived at compile time) equals the
    per-mode definition (8.3.1.2, i4_pred_px) on random neighbourhoods."""
    lib = ctypes.CDLL(EMU_LIB)
    lib.emu_i4_table_check.restype = ctypes.c_long
    assert lib.emu_i4_table_check(7, 20000) == 0


@pytest.mark.parametrize("mode", [4, 12, 5], ids=["fam3", "fam3_bad_guess", "intra_and_fam3"])
@pytest.mark.parametrize("cfg", ALL, ids=[c[0] for c in ALL])
def test_fam3_helpers_match_reference(cfg, mode):
    """Every P macroblock's 8x8-family helper task (hl_mbcore.h guess_inter
    with f3out: the P8x8 partitionings searched from the MB-start live
    TotalCoeffs, with the nC-class intervals of the entry values it read) run
    first; the macroblock takes the helper's family when its real entry state
    lies in every interval (f3_verify), else searches the family itself: the
    same streams.  mode 12 makes the helper start from wrong entry values, so
    both the rejection and the acceptance of an unread wrong value are
    exercised; mode 5 runs both kinds of helper."""
    name, w, h, n, qp, mer, db, gop, seed = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    enc = EmuEncoder(w, h, qp, mer, db, gop, GOLD[name].get("early_term", 0))
    enc.lib.emu_set_helper(ctypes.c_void_p(enc.h_), mode)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"
    kept = enc.lib.emu_helper_fam3(ctypes.c_void_p(enc.h_), 0)
    rejected = enc.lib.emu_helper_fam3(ctypes.c_void_p(enc.h_), 1)
    if any(f % gop for f in range(n)) and w * h >= 64 * 48:
        assert kept + rejected > 0


def test_kernel_logic_fails_where_reference_fails():
    """QP 8 (negative lambda): the first P picture's slice outgrows the
    reference's slice buffer; the kernel logic and the host writer refuse the
    same frame (HL_ERROR_TOOSHORT in the product) after the same bytes."""
    from hl_testlib import _planes, check_reference_failure

    def enc_ok(e, frame):
        y, u, v = _planes(frame, e.w, e.h)
        n = e.lib.emu_encode_frame(ctypes.c_void_p(e.h_), y.ctypes.data, u.ctypes.data, v.ctypes.data, e.out.ctypes.data, e.out.size)
        return e.out[:n].tobytes() if n > 0 else None

    check_reference_failure("fail_qcif_qp8_neg_lambda", lambda c: EmuEncoder(c[1], c[2], c[4], c[5], c[6], c[7]), enc_ok, GOLD)


def test_fam3_helper_entry_guess_rejections():
    """The partitioning helpers' entry guess (one coefficient in every block,
    hl_mbcore.h encode_mb) keeps their rejections low -- a speed property,
    the bytes are checked above: over three golden P-picture sequences
    11.4 % of the partitionings were rejected with it, 18.2 % with the
    address's values from the previous picture (tools/fam3_guess_stats.py)."""
    kept = rejected = 0
    for cfg in GOLDEN_CONFIGS:
        if cfg[0] not in ("cif_ippp_qp31_me8", "qcif_ippp_qp28_db", "w480_h272_qp28_me16"):
            continue
        name, w, h, n, qp, mer, db, gop, seed = cfg
        clip = golden_input(cfg)
        enc = EmuEncoder(w, h, qp, mer, db, gop)
        enc.lib.emu_set_helper(ctypes.c_void_p(enc.h_), 4)
        for f in range(n):
            enc.encode(clip[f])
        kept += enc.lib.emu_helper_fam3(ctypes.c_void_p(enc.h_), 0)
        rejected += enc.lib.emu_helper_fam3(ctypes.c_void_p(enc.h_), 1)
    assert kept + rejected > 10000
    assert rejected / (kept + rejected) < 0.13, (kept, rejected)
