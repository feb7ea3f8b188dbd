"""Spatial SVC on the GPU (hartallo_amd.SvcEncoder -> hl_amd_add_layer /
hl_amd_encode_layer, the k_svc_mb kernel) against the goldens the reference
encoder itself produced (tests/golden/make_svc_golden.py): every access
unit's bytes and every layer's reconstruction, bit-exact, including BASELINE
config 4 (480x272 / 960x544 / 1920x1088, 31 frames across the second IDR).
The layer-sharded protocol (hl_amd_set_layer_range / _export_layer /
_import_layer, hartallo_amd/svc_pipeline.py) is checked on one GPU with the
state handed over in device buffers, as RCCL does between ranks."""
import hashlib
import json
import os

import numpy as np
import pytest

from hartallo_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "svc_golden.json")))

pytestmark = pytest.mark.gpu


def md5(b) -> str:
    return hashlib.md5(b).hexdigest()


def _planes(frame, w, h):
    n = w * h
    return frame[:n], frame[n:n + n // 4], frame[n + n // 4:]


@pytest.mark.parametrize("name", sorted(GOLD))
def test_svc_gpu_matches_reference(name):
    from hartallo_amd import SvcEncoder

    g = GOLD[name]
    L, w0, h0 = g["layers"], g["w0"], g["h0"]
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, g["frames"], g["seed"])
    enc = SvcEncoder(w0, h0, L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"])
    for i in range(g["frames"]):
        out = b""
        for l in range(L):
            w, h = w0 << l, h0 << l
            r = enc.encode_layer(l, *_planes(clips[l][i], w, h))
            if r.type & 2:
                out += r.hdr
            if l == L - 1:
                assert r.type & 1
                out += b"\x00\x00\x01" + r.data
            else:
                assert not r.type & 1
        for l in range(L):
            assert md5(enc.layer_recon(l).tobytes()) == g["recon_md5"][l][i], f"AU {i} layer {l}: reconstruction differs"
        assert md5(out) == g["au_md5"][i], f"AU {i}: {len(out)} bytes vs {g['au_bytes'][i]}"
    assert enc.unpinned() == 0


@pytest.mark.parametrize("name,splits,fallback", [("c4_svc3_480x272_s41", (1, 31), False), ("svc3_64x48_qp30_gop3", (2, 3, 5), False),
                                                  ("svc2_qcif_qp36_nodb_gop2", (4,), False), ("svc3_64x48_qp30_gop3", (1, 4, 5), True),
                                                  ("c4_svc3_480x272_s41", (6,), True)])
def test_svc_gpu_layers_batch(name, splits, fallback, monkeypatch):
    """hl_amd_encode_layers_batch (frame-pipelined base layer, then the
    enhancement layers) equals the per-call stream, across batch boundaries.
    fallback: every base run is re-encoded picture by picture
    (HL_AMD_FORCE_FALLBACK), so the enhancement layers coded from the live
    run are rolled back and coded again from the final base pictures."""
    import torch

    from hartallo_amd import SvcEncoder

    if fallback:
        monkeypatch.setenv("HL_AMD_FORCE_FALLBACK", "1")

    g = GOLD[name]
    L, w0, h0 = g["layers"], g["w0"], g["h0"]
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, g["frames"], g["seed"])
    dev = [torch.from_numpy(clips[l][:splits[-1]]).cuda() for l in range(L)]
    enc = SvcEncoder(w0, h0, L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"])
    md5s, lo = [], 0
    for hi in splits:
        ptrs = []
        for l in range(L):
            n = (w0 << l) * (h0 << l)
            ptrs.append([(dev[l][i].data_ptr(), dev[l][i].data_ptr() + n, dev[l][i].data_ptr() + n + n // 4) for i in range(lo, hi)])
        for r in enc.encode_layers_batch_device(ptrs):
            md5s.append(md5(r.annexb()))
        st = enc.last_batch_stats()
        assert st["fallbacks"] == (st["runs"] if fallback else 0) and st["waits_gave_up"] == 0, st
        lo = hi
    assert md5s == g["au_md5"][:splits[-1]]
    for l in range(L):
        assert md5(enc.layer_recon(l).tobytes()) == g["recon_md5"][l][splits[-1] - 1]
    assert enc.unpinned() == 0


@pytest.mark.parametrize("ranks", [2, 3])
def test_svc_gpu_layer_sharded(ranks):
    import torch

    from hartallo_amd import SvcEncoder, svc_pipeline

    name = "svc3_64x48_qp30_gop3"
    g = GOLD[name]
    L, w0, h0 = g["layers"], g["w0"], g["h0"]
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, g["frames"], g["seed"])
    dev = [[tuple(torch.from_numpy(np.ascontiguousarray(p)).cuda() for p in _planes(clips[l][i], w0 << l, h0 << l))
            for i in range(g["frames"])] for l in range(L)]
    ranges = svc_pipeline.layer_ranges(L, ranks)
    encs = [svc_pipeline.GpuLayerAdapter(SvcEncoder(w0, h0, L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"],
                                                    first=a, last=b), dev) for a, b in ranges]
    parts = [[] for _ in ranges]
    for t in range(g["frames"]):
        buf = None
        for r, (a, b) in enumerate(ranges):
            if r:
                encs[r].import_layer(a - 1, buf)
            hdr, part = b"", None
            for l in range(a, b + 1):
                h, p = encs[r].encode(l, t)
                hdr += h
                if p is not None:
                    part = p
            parts[r].append((hdr, part))
            buf = torch.empty(encs[r].layer_state_bytes(b), dtype=torch.uint8, device="cuda")
            encs[r].export_layer(b, buf)
    aus = svc_pipeline.assemble(parts)
    assert [md5(a) for a in aus] == g["au_md5"]


def test_svc_api_errors():
    from hartallo_amd import HlAmdError, SvcEncoder
    from hartallo_amd._lib import (HL_AMD_ERROR_INVALID_PARAMETER, HL_AMD_ERROR_INVALID_STATE, HL_AMD_ERROR_NOT_FOUND,
                                   HL_AMD_ERROR_NOT_IMPLEMENTED)

    enc = SvcEncoder(64, 48, 2)
    z = lambda n: np.zeros(n, np.uint8)  # noqa: E731
    # layers come base first within an access unit (INVALID_STATE)
    with pytest.raises(HlAmdError) as ei:
        enc.encode_layer(1, z(128 * 96), z(64 * 48), z(64 * 48))
    assert ei.value.code == HL_AMD_ERROR_INVALID_STATE
    # a frame of no layer's size (hl_codec_264.c:478-481)
    r = enc.lib.hl_amd_encode_layer(enc._h, 96, 48, z(96 * 48).ctypes.data, z(96 * 12).ctypes.data, z(96 * 12).ctypes.data, 0,
                                    None)
    assert r == HL_AMD_ERROR_INVALID_PARAMETER  # null result
    from hartallo_amd._lib import _Result
    import ctypes
    res = _Result()
    a, b = z(96 * 48), z(96 * 12)
    assert enc.lib.hl_amd_encode_layer(enc._h, 96, 48, a.ctypes.data, b.ctypes.data, b.ctypes.data, 0, ctypes.byref(res)) == \
        HL_AMD_ERROR_NOT_FOUND
    base = SvcEncoder(64, 48, 1)
    assert base.lib.hl_amd_add_layer(base._h, 192, 144) == HL_AMD_ERROR_INVALID_PARAMETER  # ratio 3 (hl_codec.c:113-121)
    assert base.lib.hl_amd_add_layer(base._h, 256, 192) == HL_AMD_ERROR_NOT_IMPLEMENTED    # ratio 4: only dyadic layers
    assert base.lib.hl_amd_add_layer(base._h, 32, 32) == HL_AMD_ERROR_INVALID_PARAMETER    # decreasing (hl_codec.c:107-112)
