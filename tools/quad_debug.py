"""Development: print the first blocks where the quad pipeline (hl_quad.h)
differs from the scalar primitives (tests/gpu_unit/libhl_unit.so)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_unit import FIELDS, LIB, _blocks  # noqa: E402

lib = ctypes.CDLL(LIB)
np.set_printoptions(linewidth=200)
for qp in (0, 28):
    for mode in (0, 2):
        n = 4096
        src, pred = _blocks(n, 1000 * qp + mode)
        outs = []
        for coop in (0, 2):
            o = np.zeros((n, FIELDS), dtype=np.int32)
            lib.unit_run(src.ctypes.data_as(ctypes.c_void_p), pred.ctypes.data_as(ctypes.c_void_p), n, qp, mode, coop, o.ctypes.data_as(ctypes.c_void_p))
            outs.append(o)
        bad = np.nonzero((outs[0] != outs[1]).any(axis=1))[0]
        print(f"qp {qp} mode {mode}: {bad.size} differ")
        for b in bad[:3]:
            print(" res ", (src[b].astype(int) - pred[b]).tolist())
            print(" scal", outs[0][b][:21].tolist())
            print(" quad", outs[1][b][:21].tolist())
            print(" rec s", outs[0][b][21:].tolist(), "q", outs[1][b][21:].tolist())
