"""Model check of the pipelined-run schedule (hartallo_amd/csrc/hl_pipeline.h),
through the C++ trigger rules themselves (exported by the host build of the
kernel logic, tests/emu/libhl_emu.so).

Each macroblock task decides its MB, then deblocks and computes the
quarter-pel planes of the blocks whose trigger it is.  Tasks run in random
orders consistent with the wavefront dependencies (MB (x, y) after (x-1, y)
and (x+1, y-1)); the checks:
  1. deblock(X, Y) after deblock(X-1, Y), deblock(X, Y-1), deblock(X+1, Y-1):
     the reference's raster deblocking order (deblock.c) as far as the
     filtered samples overlap;
  2. deblock(X, Y) after the decision of every MB whose intra prediction reads
     samples it modifies (intra prediction reads unfiltered samples: the
     reference deblocks after the whole picture, slice.c:1868-1880);
  3. planes(X, Y) after the deblocking of its 3x3 neighbourhood (6-tap reach);
  4. every deblock and plane block exactly once.
"""
import ctypes
import random

import pytest

from hl_testlib import emu_lib


def _blocks(lib, kind, x, y, mbw, mbh):
    out = (ctypes.c_int * 64)()
    n = lib.emu_task_blocks(kind, x, y, mbw, mbh, out)
    return [(out[2 * i], out[2 * i + 1]) for i in range(n)]


def _deps(x, y, mbw):
    d = []
    if x > 0:
        d.append((x - 1, y))
    if y > 0:
        d.append((x + 1, y - 1) if x + 1 < mbw else (x, y - 1))
    return d


@pytest.mark.parametrize("mbw,mbh", [(1, 1), (2, 1), (1, 2), (2, 2), (3, 3), (4, 2), (2, 4), (5, 7), (11, 9), (22, 18), (8, 3)])
def test_task_schedule(mbw, mbh):
    lib = emu_lib()
    lib.emu_task_blocks.argtypes = [ctypes.c_int] * 5 + [ctypes.POINTER(ctypes.c_int)]
    tdb = {(x, y): _blocks(lib, 0, x, y, mbw, mbh) for y in range(mbh) for x in range(mbw)}
    tpl = {(x, y): _blocks(lib, 1, x, y, mbw, mbh) for y in range(mbh) for x in range(mbw)}
    inside = lambda p: 0 <= p[0] < mbw and 0 <= p[1] < mbh  # noqa: E731
    for seed in range(12):
        rng = random.Random(seed)
        done, order, pending = set(), [], [(x, y) for y in range(mbh) for x in range(mbw)]
        while pending:
            t = rng.choice([p for p in pending if all(d in done for d in _deps(*p, mbw))])
            pending.remove(t)
            done.add(t)
            order.append(t)
        decided, deblocked, planed = set(), set(), set()
        for t in order:
            decided.add(t)
            for (X, Y) in tdb[t]:
                for p in [(X - 1, Y), (X, Y - 1), (X + 1, Y - 1)]:
                    assert not inside(p) or p in deblocked, ("deblock order", (X, Y), p, t)
                for r in [(X + 1, Y), (X - 1, Y + 1), (X, Y + 1), (X + 1, Y + 1), (X - 2, Y + 1)]:
                    assert not inside(r) or r in decided, ("unfiltered reader pending", (X, Y), r, t)
                assert (X, Y) not in deblocked
                deblocked.add((X, Y))
            for (X, Y) in tpl[t]:
                for a in range(X - 1, X + 2):
                    for b in range(Y - 1, Y + 2):
                        assert not inside((a, b)) or (a, b) in deblocked, ("planes", (X, Y), (a, b), t)
                assert (X, Y) not in planed
                planed.add((X, Y))
        assert len(deblocked) == len(planed) == mbw * mbh
