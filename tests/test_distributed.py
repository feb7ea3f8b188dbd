"""world_size-2 gloo tests of the multi-stream plumbing bench.py uses (BASELINE
config 5: one independent stream per rank, no data-path collective): every
rank joins, ranks encode different streams, the reported time is the max
over ranks, the whole-job frame count is world * steps, and the bit-exact
flag is the minimum over ranks."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from hartallo_amd import dist, synth

    r, w, local = dist.init_from_env()
    elapsed = 1.0 + r  # rank 1 is the slowest
    dist.barrier()
    m = dist.max_over_ranks(elapsed)
    clip = synth.clip(32, 16, 2, dist.stream_seed(r))
    q.put((r, w, local, m, int(clip.sum())))
    dist.shutdown()


def _encode_worker(rank, world, port, q):
    """Each rank encodes its own stream (its own seed, dist.stream_seed) with
    the host build of the kernel logic (tests/emu) and checks every frame
    against the CPU oracle; the ranks then combine as bench.py does."""
    import sys

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from hl_testlib import EmuEncoder, OracleEncoder

    from hartallo_amd import dist, synth

    r, w, _ = dist.init_from_env()
    W, H, n = 64, 48, 4
    clip = synth.clip(W, H, n, dist.stream_seed(r))
    e, o = EmuEncoder(W, H, 28, 16, 1, 3), OracleEncoder(W, H, 28, 16, 1, 3)
    import hashlib

    ok, h = True, hashlib.md5()
    for f in range(n):
        a, b = e.encode(clip[f]), o.encode(clip[f])
        ok = ok and a == b
        h.update(a)
    exact = dist.min_over_ranks(1 if ok else 0)
    frames = dist.sum_over_ranks([n])[0]
    q.put((r, exact, frames, h.hexdigest()))
    dist.shutdown()


def test_two_rank_gloo_streams_encode():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_encode_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1]
    assert all(r[1] == 1 for r in res), res  # every rank's stream bit-exact against the oracle
    assert all(r[2] == 2 * 4 for r in res)  # whole-job frame count
    assert res[0][3] != res[1][3]  # different streams per rank


def test_two_rank_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == [0, 1]
    assert all(r[1] == world and r[3] == pytest.approx(2.0) for r in res)
    assert res[0][4] != res[1][4]  # different streams per rank
