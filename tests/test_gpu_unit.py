"""GPU unit parity of the cooperative 4x4 pipelines -- 16-lane rows (hl_coop.h)
and 4-lane quads (hl_quad.h, the candidate evaluation): DPP transforms,
quantisation, mask-based CAVLC statistics -- against the scalar
primitives (hl_prims.h, the restatement of transf.c / quant.c /
residual.c) on the same random blocks.  Bit-exact: every field must match.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gpu_unit", "libhl_unit.so")
FIELDS = 5 + 32  # tc, t1, rest, sctr, dist, q[16], rec[16]


def _blocks(n, seed):
    rng = np.random.default_rng(seed)
    pred = rng.integers(0, 256, (n, 16), dtype=np.int32)
    kind = rng.integers(0, 4, n)
    amp = np.choose(kind, [2, 6, 30, 255])
    res = (rng.integers(-255, 256, (n, 16)) * amp[:, None]) // 255
    # sparse residuals: most coefficients zero
    res[kind == 0] *= rng.integers(0, 2, (int((kind == 0).sum()), 16))
    src = np.clip(pred + res, 0, 255)
    return src.astype(np.uint8), pred.astype(np.uint8)


@pytest.mark.parametrize("mode", [0, 1, 2], ids=["inter", "intra", "ac"])
@pytest.mark.parametrize("qp", [0, 6, 12, 20, 28, 36, 44, 51])
def test_coop_block_pipeline(gpu, qp, mode):
    lib = ctypes.CDLL(LIB)
    assert lib.unit_sizeof_out() == 4 * FIELDS
    n = 4096
    src, pred = _blocks(n, 1000 * qp + mode)
    outs = []
    for coop in (0, 1, 2):
        o = np.zeros((n, FIELDS), dtype=np.int32)
        rc = lib.unit_run(src.ctypes.data_as(ctypes.c_void_p), pred.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(n), ctypes.c_int(qp),
                          ctypes.c_int(mode), ctypes.c_int(coop), o.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0
        outs.append(o)
    for k, name in ((1, "coop"), (2, "quad")):
        bad = np.nonzero((outs[0] != outs[k]).any(axis=1))[0]
        assert bad.size == 0, f"{name}: {bad.size} blocks differ; first {bad[0]}: scalar {outs[0][bad[0]][:5]} {name} {outs[k][bad[0]][:5]}"


@pytest.mark.parametrize("w,h", [(32, 16), (176, 144), (352, 288), (1920, 1088)])
def test_planes_kernel(gpu, w, h):
    """k_planes (hl_filters.h) against the per-sample definition
    qpel_plane_sample (interpol.c:74-225 edge semantics) on a random picture."""
    lib = ctypes.CDLL(LIB)
    rng = np.random.default_rng(w + h)
    ref = rng.integers(0, 256, (h, w), dtype=np.uint8)
    pstride = (w + 80 + 63) & ~63
    size = 4 * pstride * (h + 80)
    a, b = np.zeros(size, np.uint8), np.zeros(size, np.uint8)
    assert lib.unit_planes(ref.ctypes.data_as(ctypes.c_void_p), w, h, a.ctypes.data_as(ctypes.c_void_p), b.ctypes.data_as(ctypes.c_void_p)) == 0
    bad = np.nonzero(a != b)[0]
    assert bad.size == 0, f"{bad.size} samples differ; first at plane {bad[0] // (size // 4)}"
