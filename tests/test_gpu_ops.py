"""Op-level parity of the gfx950 kernels against the reference's OWN per-block
kernels (fixture kind 1).

tests/golden/ops_*.npz hold seeded inputs and the outputs of the reference's
functions (oracle/_ref/ref_ops, built from /root/reference's sources; made
by tests/golden/make_op_golden.py):
  ops_xform  transf_frw_residual4x4 + quant_frw4x4_scale_ac +
             quant_scale_residual4x4 + transf_inverse_residual4x4
             (transf.c:376-458, 716-772; quant.c:68-139), every QP, inter /
             intra rounding
  ops_cavlc  hl_codec_264_residual_write_block_cavlc (residual.c:587-901):
             the written bits, luma 4x4 / Intra16x16 AC / chroma AC at nC
             0..16, chroma DC (nC -1), and the AC lists as the RDO prices
             them (0, 15, 16: rdo.c:1676)
  ops_lpred  hl_codec_264_interpol_luma (pred_inter.c:339-885): 16x16
             predictions, all 16 quarter-pel phases, interior and edge
             macroblocks, motion up to 24 samples outside the picture
  ops_dblk   the baseline u8 edge filter (deblock.c:1836-2420: indexA /
             alpha / beta, get_threshold8samples, filter8samples0 bs < 4 /
             bs == 4), bS 1..4 x indexA 0..51, luma and chroma
and the product's device code runs on the same inputs through
tests/gpu_unit/libhl_unit.so: the quad pipeline of the candidate evaluation
and the 16-lane rows of the intra decisions (hl_quad.h, hl_coop.h),
cavlc_block (hl_cavlc.h) and quad_cavlc's rate, k_planes + the finalize's
quarter-pel sample pairs (hl_filters.h, hl_mbcore.h), deblock_line
(hl_filters.h).  Bit-exact: everything is integer.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "gpu_unit", "libhl_unit.so")
GOLD = os.path.join(HERE, "golden")


def _lib():
    return ctypes.CDLL(LIB)


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _gold(name):
    return np.load(os.path.join(GOLD, f"ops_{name}.npz"))


@pytest.mark.parametrize("coop", [2, 1, 0], ids=["quad", "rows16", "scalar"])
def test_transform_quant_idct_vs_reference(gpu, coop):
    """Levels (raster) and reconstruction of every block at every QP, inter
    and intra rounding, against the reference's transform / quantiser /
    dequantiser / IDCT."""
    g = _gold("xform")
    lib = _lib()
    fields = 5 + 32
    assert lib.unit_sizeof_out() == 4 * fields
    bad = []
    for qp in range(52):
        for intra in (0, 1):
            m = (g["qp"] == qp) & (g["intra"] == intra)
            src, pred = np.ascontiguousarray(g["src"][m]), np.ascontiguousarray(g["pred"][m])
            n = len(src)
            o = np.zeros((n, fields), np.int32)
            assert lib.unit_run(_ptr(src), _ptr(pred), n, qp, intra, coop, _ptr(o)) == 0
            dq = np.nonzero((o[:, 5:21] != g["q"][m]).any(axis=1))[0]
            dr = np.nonzero((o[:, 21:37] != g["rec"][m]).any(axis=1))[0]
            if dq.size or dr.size:
                bad.append((qp, intra, dq.size, dr.size))
    assert not bad, f"(qp, intra, blocks with other levels, blocks with another reconstruction): {bad[:8]}"


def _cavlc_out():
    return np.dtype([("nbits", "<i4"), ("quad_bits", "<i4"), ("tc", "<i4"), ("pad", "<i4"), ("words", "<u4", 24)])


def test_cavlc_bits_vs_reference(gpu):
    """The GPU residual writer (cavlc_block) writes the reference's bits, and
    the candidate evaluation's rate (quad_cavlc) is the reference's bit count
    of every coded luma 4x4 / Intra16x16 AC block at the nC class it reads."""
    g = _gold("cavlc")
    lib = _lib()
    dt = _cavlc_out()
    assert lib.unit_sizeof_cavlc_out() == dt.itemsize
    n = len(g["kind"])
    cin = np.zeros(n, np.dtype([("kind", "<i4"), ("nC", "<i4"), ("level", "<i4", 16)]))
    cin["kind"], cin["nC"], cin["level"] = g["kind"], g["nC"], g["level"]
    out = np.zeros(n, dt)
    assert lib.unit_cavlc(_ptr(cin), n, _ptr(out)) == 0
    # the bits themselves: the product's big-endian words against the reference's bytes
    got = out["words"].astype(">u4").view(np.uint8).reshape(n, 96)
    nb = g["nbits"]
    assert np.array_equal(out["nbits"], nb), f"bit counts differ at {np.nonzero(out['nbits'] != nb)[0][:8]}"
    mask = (np.arange(96 * 8)[None, :] < nb[:, None]).reshape(n, 96, 8)
    gb = np.unpackbits(g["bits"], axis=1).reshape(n, 96, 8) & mask
    pb = np.unpackbits(got, axis=1).reshape(n, 96, 8) & mask
    diff = np.nonzero((gb != pb).any(axis=(1, 2)))[0]
    assert diff.size == 0, f"{diff.size} blocks written differently; first {diff[0]} (kind {g['kind'][diff[0]]}, nC {g['nC'][diff[0]]})"
    # the RDO's rate: coded blocks of kinds 0 / 4 (the reference prices AC lists
    # as 16-entry blocks, rdo.c:1676; an uncoded block costs no rate there)
    k = ((g["kind"] == 0) | (g["kind"] == 4)) & (out["tc"] > 0)
    assert k.sum() > 1000
    d = np.nonzero(k & (out["quad_bits"] != nb))[0]
    assert d.size == 0, f"quad_cavlc rate differs for {d.size} blocks; first {d[:4]} (kinds {g['kind'][d[:4]]}, nC {g['nC'][d[:4]]})"


def test_luma_interpolation_vs_reference(gpu):
    """16x16 predictions at every quarter-pel phase and macroblock of a 96x64
    picture, motion clamped at the picture edges, against the reference's
    hl_codec_264_interpol_luma."""
    g = _gold("lpred")
    lib = _lib()
    W, H = int(g["W"]), int(g["H"])
    n = len(g["mbx"])
    pin = np.zeros(n, np.dtype([("mbx", "<i4"), ("mby", "<i4"), ("mvx", "<i4"), ("mvy", "<i4")]))
    for k in ("mbx", "mby", "mvx", "mvy"):
        pin[k] = g[k]
    luma = np.ascontiguousarray(g["luma"])
    out = np.zeros((n, 16, 16), np.uint8)
    assert lib.unit_lpred(_ptr(luma), W, H, _ptr(pin), n, _ptr(out)) == 0
    bad = np.nonzero((out != g["pred"]).any(axis=(1, 2)))[0]
    assert bad.size == 0, (f"{bad.size} predictions differ; first: mb ({g['mbx'][bad[0]]}, {g['mby'][bad[0]]}) "
                           f"mv ({g['mvx'][bad[0]]}, {g['mvy'][bad[0]]})")


def test_deblock_lines_vs_reference(gpu):
    """8-line edge segments at every bS 1..4 x indexA 0..51, luma and chroma,
    against the reference's baseline filter steps (thresholds, Table 8-16 /
    8-17, bS < 4 and bS == 4 filters, bypass of unfiltered lines)."""
    g = _gold("dblk")
    lib = _lib()
    n = len(g["bS"])
    din = np.zeros(n, np.dtype([("p", "u1", (4, 8)), ("q", "u1", (4, 8)), ("bS", "<i4"), ("indexA", "<i4"), ("chroma", "<i4")]))
    din["p"], din["q"], din["bS"], din["indexA"], din["chroma"] = g["p_in"], g["q_in"], g["bS"], g["indexA"], g["chroma"]
    out = np.zeros(n, np.dtype([("p", "u1", (3, 8)), ("q", "u1", (3, 8))]))
    assert lib.unit_dblk(_ptr(din), n, _ptr(out)) == 0
    changed = (g["p_out"] != g["p_in"][:, :3]).any(axis=(1, 2))
    assert changed.sum() > n // 4  # the vectors do reach the filters
    bad = np.nonzero((out["p"] != g["p_out"]).any(axis=(1, 2)) | (out["q"] != g["q_out"]).any(axis=(1, 2)))[0]
    assert bad.size == 0, (f"{bad.size} segments differ; first: bS {g['bS'][bad[0]]} indexA {g['indexA'][bad[0]]} "
                           f"chroma {g['chroma'][bad[0]]}")
