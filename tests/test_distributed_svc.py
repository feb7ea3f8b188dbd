"""Layer-sharded spatial SVC across processes (hartallo_amd/svc_pipeline.py,
BASELINE config 4) on the CPU: gloo world sizes 2 and 3, each rank coding its
layer range with the host build of the kernel logic (tests/emu) and handing
the layer state to the next rank with point-to-point sends.  The stream the
ranks assemble must equal the reference encoder's (tests/golden/svc_golden.json)."""
import hashlib
import json
import os
import socket

import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "svc_golden.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _EmuAdapter:
    def __init__(self, enc, clips):
        self.enc, self.clips = enc, clips

    def encode(self, layer, t):
        o = self.enc.encode(layer, self.clips[layer][t])
        k = self.enc.last_hdr()
        return o[:k], (o[k + 3:] if len(o) > k else None)

    def layer_state_bytes(self, layer):
        return self.enc.layer_state_bytes(layer)

    def export_layer(self, layer, buf):
        buf.numpy()[:] = self.enc.export_layer(layer)

    def import_layer(self, layer, buf):
        self.enc.import_layer(layer, buf.numpy())


def _worker(rank, world, port, name, q):
    import sys

    sys.path.insert(0, HERE)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch
    import torch.distributed as dist

    from hartallo_amd import synth, svc_pipeline
    from hl_testlib import EmuSvcEncoder

    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = GOLD[name]
    L = g["layers"]
    role = svc_pipeline.role_of(rank, world, L)
    clips = synth.svc_clips(g["w0"] << (L - 1), g["h0"] << (L - 1), L, g["frames"], g["seed"])
    enc = EmuSvcEncoder(g["w0"], g["h0"], L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"])
    enc.set_range(role.first, role.last)
    parts = svc_pipeline.run_access_units(_EmuAdapter(enc, clips), role, None, g["frames"], dist,
                                          lambda nb: torch.zeros(nb, dtype=torch.uint8))
    allp = [None] * world
    dist.all_gather_object(allp, parts)
    if rank == 0:
        group = [allp[r] for r in range(world) if svc_pipeline.role_of(r, world, L).group == role.group]
        aus = svc_pipeline.assemble(group)
        q.put([hashlib.md5(a).hexdigest() for a in aus])
    dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "svc3_64x48_qp30_gop3"), (3, "svc3_64x48_qp30_gop3"), (2, "svc2_qcif_qp36_nodb_gop2")])
def test_layer_sharded_stream_equals_reference(world, name):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in ps:
        p.start()
    md5s = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert md5s == GOLD[name]["au_md5"]


def test_layer_ranges():
    from hartallo_amd.svc_pipeline import layer_ranges, role_of

    assert layer_ranges(3, 1) == [(0, 2)]
    assert layer_ranges(3, 2) == [(0, 0), (1, 2)]
    assert layer_ranges(3, 3) == [(0, 0), (1, 1), (2, 2)]
    assert layer_ranges(3, 8) == [(0, 0), (1, 1), (2, 2)]
    # 4 ranks, 3 layers: one 3-rank stream, one whole stream on rank 3
    roles = [role_of(r, 4, 3) for r in range(4)]
    assert [(x.group, x.first, x.last, x.prev, x.next) for x in roles] == [(0, 0, 0, -1, 1), (0, 1, 1, 0, 2), (0, 2, 2, 1, -1),
                                                                           (1, 0, 2, -1, -1)]
    # 8 ranks: two 3-rank streams and two whole streams
    assert [role_of(r, 8, 3).group for r in range(8)] == [0, 0, 0, 1, 1, 1, 2, 3]
