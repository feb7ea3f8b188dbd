"""Spatial SVC: the host build of the gfx950 kernel logic (tests/emu, the
product's hl_svc.h / hl_mbcore.h compiled for one lane) against the goldens
the reference encoder itself produced (tests/golden/make_svc_golden.py):
every access unit's bytes and every layer's reconstruction, bit-exact."""
import hashlib
import json
import os

import numpy as np
import pytest

from hl_testlib import EmuSvcEncoder, first_diff

from hartallo_amd import synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "svc_golden.json")))
# CPU budget: the BASELINE-sized workload is checked on its first access units
CPU_AUS = {"c4_svc3_480x272_s41": 3}


def md5(b) -> str:
    return hashlib.md5(b).hexdigest()


@pytest.mark.parametrize("name", sorted(GOLD))
def test_svc_matches_reference(name):
    g = GOLD[name]
    L, w0, h0 = g["layers"], g["w0"], g["h0"]
    n = CPU_AUS.get(name, g["frames"])
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, g["frames"], g["seed"])
    enc = EmuSvcEncoder(w0, h0, L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"])
    stream = open(os.path.join(HERE, "golden", g["stream"]), "rb").read() if g["stream"] else None
    out = b""
    for i in range(n):
        au = b"".join(enc.encode(l, clips[l][i]) for l in range(L))
        for l in range(L):
            assert md5(enc.recon(l).tobytes()) == g["recon_md5"][l][i], f"AU {i} layer {l}: reconstruction differs"
        if stream is not None and md5(au) != g["au_md5"][i]:
            pos = len(out)
            ref = stream[pos:pos + g["au_bytes"][i]]
            pytest.fail(f"AU {i}: {len(au)} vs {len(ref)} bytes, first difference at byte {first_diff(au, ref)}")
        assert md5(au) == g["au_md5"][i], f"AU {i}: bytes differ ({len(au)} vs {g['au_bytes'][i]})"
        out += au
    assert enc.unpinned() == 0


def test_svc_inputs_are_layered():
    # each layer is the 2x2 box-average downscale of the one above
    cl = synth.svc_clips(64, 32, 2, 1, 1)
    top = cl[1][0][:64 * 32].reshape(32, 64).astype(np.int32)
    low = cl[0][0][:32 * 16].reshape(16, 32)
    exp = (top[0::2, 0::2] + top[0::2, 1::2] + top[1::2, 0::2] + top[1::2, 1::2] + 2) >> 2
    assert np.array_equal(low, exp)
