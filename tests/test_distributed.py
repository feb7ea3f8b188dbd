"""world_size-2 gloo test of the multi-stream plumbing bench.py uses: every
rank joins, ranks encode different streams, the reported time is the max
over ranks and the whole-job frame count is world * steps."""
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
