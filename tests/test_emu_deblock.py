"""The tiled deblocking of the GPU -- the row kernel k_deblock_rows
(hl_filters.h DbTile helpers, run lane by lane in the tightest order the
kernel's waits allow, tests/emu/hl_emu.hip deblock_rows_emu) and the per-MB
LDS tiles of k_pipeline's tasks (DbMbTile, in the pipelined schedule's task
order, deblock_tasks_emu) -- against the per-MB raster filter
(deblock_mb_step, the reference's order, deblock.c:192-284): random samples
with steps at block edges and random MB objects (intra, skip, every
partition shape, coded blocks, motion), so that every bS and filter branch
occurs.  Bit-exact."""
import ctypes

import pytest

from hl_testlib import emu_lib


@pytest.mark.parametrize("mode", [0, 1], ids=["rows", "tasks"])
@pytest.mark.parametrize("w,h", [(16, 16), (64, 48), (176, 144), (480, 272)])
@pytest.mark.parametrize("qp", [22, 28, 40, 51])
def test_tiled_deblock_equals_raster(w, h, qp, mode):
    lib = emu_lib()
    lib.emu_deblock_selftest.restype = ctypes.c_long
    lib.emu_deblock_selftest.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint, ctypes.c_int]
    for seed in range(3):
        assert lib.emu_deblock_selftest(w, h, qp, seed, mode) == 0, (w, h, qp, seed)
