"""The CPU oracle (oracle/hl_oracle.c) is pinned to the reference: it must
reproduce every golden stream (produced by the reference encoder itself,
tests/golden/make_golden.py) byte for byte, and its reconstructed pictures
must match the reference's per-frame MD5s."""
import json
import os

import pytest

from hl_testlib import GOLDEN, GOLDEN_CONFIGS, OracleEncoder, first_diff, golden_input, md5

GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


@pytest.mark.parametrize("cfg", GOLDEN_CONFIGS, ids=[c[0] for c in GOLDEN_CONFIGS])
def test_oracle_matches_reference(cfg):
    name, w, h, n, qp, mer, db, gop, seed = cfg
    clip = golden_input(cfg)
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    assert md5(ref) == GOLD[name]["stream_md5"]
    enc = OracleEncoder(w, h, qp, mer, db, gop)
    out = b""
    for f in range(n):
        out += enc.encode(clip[f])
        assert md5(enc.recon()) == GOLD[name]["recon_md5"][f], f"{name}: recon of frame {f}"
    assert out == ref, f"{name}: first differing byte {first_diff(out, ref)}"
    assert enc.rdo_overflows() == 0


def test_oracle_rejects_unsupported():
    with pytest.raises(ValueError):
        OracleEncoder(1920, 1080)  # height not a multiple of 16 (hl_codec_264.c:437)
