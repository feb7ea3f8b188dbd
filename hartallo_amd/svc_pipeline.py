"""Layer-sharded spatial SVC over several processes (BASELINE config 4).

The reference codes the layers of an access unit one after the other in one
hl_codec_t (hl_codec_264.c:404-1017; test_encoder.c:171-202 calls
hl_codec_encode once per layer, base first).  Enhancement layer l needs, of
its access unit, only layer l-1's reconstructed picture and macroblock
objects (hartallo_amd/csrc/hl_svc.h), so the layers pipeline across ranks:
rank r codes a contiguous range of layers, then hands the top layer's state
(hl_amd_export_layer: picture Y|U|V + MbState[], ~1.5 B/px + 428 B/MB) to
rank r + 1 with one point-to-point send -- RCCL over xGMI with the "nccl"
backend, gloo on the CPU -- and rank r + 1 imports it (hl_amd_import_layer)
before coding its own range.  While rank r + 1 codes access unit t, rank r
already codes t + 1; the state buffers are double-buffered so that a send
still in flight never sees the next access unit's export.

The base layer (the full RDO search, hl_mbcore.h) dominates the cost, so it
gets a rank of its own and the enhancement layers (no search) share the rest.
Ranks beyond what one stream's layers can use run further streams.
"""
from __future__ import annotations

from dataclasses import dataclass


def layer_ranges(layers: int, ranks: int):
    """[first, last] per rank of one stream's group: the base layer alone on
    rank 0, the enhancement layers split as evenly as possible over the rest."""
    if ranks <= 1:
        return [(0, layers - 1)]
    ranks = min(ranks, layers)
    out = [(0, 0)]
    rest, k = layers - 1, ranks - 1
    a = 1
    for i in range(k):
        n = rest // k + (1 if i < rest % k else 0)
        out.append((a, a + n - 1))
        a += n
    return out


@dataclass
class Role:
    group: int      # stream index
    group_rank: int  # position of this rank in its stream's layer pipeline
    group_size: int
    first: int
    last: int
    prev: int       # global rank coding the layers below (-1: none)
    next: int       # global rank coding the layers above (-1: none)
    leader: int     # global rank of the group's base layer (collects the stream)


def role_of(rank: int, world: int, layers: int) -> Role:
    """Groups of min(layers, world) consecutive ranks each code one stream
    layer-sharded; leftover ranks code a whole stream each."""
    g = min(layers, world)
    full = (world // g) * g
    if rank < full:
        group, gr, size = rank // g, rank % g, g
    else:
        group, gr, size = world // g + (rank - full), 0, 1
    first, last = layer_ranges(layers, size)[gr]
    base = rank - gr
    return Role(group, gr, size, first, last, rank - 1 if gr > 0 else -1, rank + 1 if gr < size - 1 else -1, base)


def run_access_units(enc, role: Role, frames, n: int, dist, make_buffer, on_au=None):
    """Codes n access units of one stream on this rank.

    enc         encoder adapter: encode(layer, au) -> (hdr: bytes, part: bytes|None),
                export_layer(layer, buf), import_layer(layer, buf), layer_state_bytes(layer)
    frames      unused by this function (the adapter owns the input); kept for symmetry
    dist        torch.distributed (initialised) or None for a single rank
    make_buffer make_buffer(nbytes) -> tensor used for the exchanged state
    Returns [(hdr bytes of the AU's calls, this rank's part of the AU)] per AU.
    """
    out = []
    bufs_in = bufs_out = None
    if role.prev >= 0:
        bufs_in = [make_buffer(enc.layer_state_bytes(role.first - 1)) for _ in range(2)]
    if role.next >= 0:
        bufs_out = [make_buffer(enc.layer_state_bytes(role.last)) for _ in range(2)]
    pending = [None, None]
    for t in range(n):
        if bufs_in is not None:
            b = bufs_in[t & 1]
            dist.recv(b, src=role.prev)
            enc.import_layer(role.first - 1, b)
        hdr, part = b"", None
        for l in range(role.first, role.last + 1):
            h, p = enc.encode(l, t)
            hdr += h
            if p is not None:
                part = p
        if bufs_out is not None:
            k = t & 1
            if pending[k] is not None:
                pending[k].wait()
            enc.export_layer(role.last, bufs_out[k])
            pending[k] = dist.isend(bufs_out[k], dst=role.next)
        out.append((hdr, part))
        if on_au is not None:
            on_au(t)
    for w in pending:
        if w is not None:
            w.wait()
    return out


def assemble(parts_by_rank):
    """The stream the reference harness writes (oracle/ref_svc_harness.c):
    per access unit the header bytes of every call (in layer order), then
    "00 00 01" and the ranks' parts joined with "00 00 01".
    parts_by_rank: [[(hdr, part) per AU] per rank of the group, in layer order]."""
    out = []
    for t in range(len(parts_by_rank[0])):
        hdr = b"".join(r[t][0] for r in parts_by_rank)
        au = b"\x00\x00\x01".join(r[t][1] for r in parts_by_rank)
        out.append(hdr + b"\x00\x00\x01" + au)
    return out


class GpuLayerAdapter:
    """hartallo_amd.SvcEncoder behind run_access_units: inputs resident in HBM
    (torch uint8 tensors per layer and access unit), exchange buffers are
    torch device tensors (RCCL reads / writes them in place)."""

    def __init__(self, enc, planes):
        self.enc = enc
        self.planes = planes  # planes[layer][au] = (y, u, v) device tensors

    def encode(self, layer, t):
        y, u, v = self.planes[layer][t % len(self.planes[layer])]
        r = self.enc.encode_layer_device(layer, y.data_ptr(), u.data_ptr(), v.data_ptr())
        return r.hdr, (r.data if r.type & 1 else None)

    def layer_state_bytes(self, layer):
        return self.enc.layer_state_bytes(layer)

    def export_layer(self, layer, buf):
        import torch

        torch.cuda.current_stream().synchronize()  # an earlier send of this buffer has finished
        self.enc.export_layer(layer, buf.data_ptr())

    def import_layer(self, layer, buf):
        import torch

        torch.cuda.current_stream().synchronize()  # the received bytes are complete
        self.enc.import_layer(layer, buf.data_ptr())
