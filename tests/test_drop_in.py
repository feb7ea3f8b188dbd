"""The drop-in boundary exercised through the reference itself.

integration/hl_codec_264_gfx950.c is the plugin a maintainer adds to
hartallo: it registers in place of the stock H.264 plugin and forwards the
encode slot (hl_codec.h:173-184) to libhartallo_amd.so.  oracle/Makefile
compiles it against the reference's own headers and links it with the
reference's own library (oracle/_ref/libhl.a) into oracle/_ref/drop_in_enc,
which encodes through hl_codec_encode exactly as source/test_encoder.c does
(oracle/drop_in_harness.c).  On the GPU its streams must equal the streams
the stock reference encoder produced (tests/golden), byte for byte --
including the early-termination goldens encoded with the hl_codec_create
default me_early_term_flag = 1 left untouched.
"""
import json
import os
import subprocess
import tempfile

import pytest

from hl_testlib import GOLDEN, GOLDEN_CONFIGS, GOLDEN_ET_CONFIGS, GOLDEN_MRF_CONFIGS, GOLDEN_RC_CONFIGS, ROOT, first_diff, golden_input

DROP_IN = os.path.join(ROOT, "oracle", "_ref", "drop_in_enc")
DROP_IN_DEC = os.path.join(ROOT, "oracle", "_ref", "drop_in_dec")
REF_DEC = os.path.join(ROOT, "oracle", "_ref", "ref_dec")
PLUGIN = os.path.join(ROOT, "integration", "hl_codec_264_gfx950.c")
REF = "/root/reference"
GOLD = json.load(open(os.path.join(GOLDEN, "golden.json")))


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")), reason="reference sources are only in the build container")
def test_plugin_compiles_against_reference_headers():
    prelude = os.path.join(ROOT, "oracle", "_ref", "prelude.h")
    cmd = ["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror=incompatible-pointer-types", "-Werror=int-conversion",
           "-Werror=implicit-function-declaration", "-D_GNU_SOURCE", "-include", "limits.h", "-include", prelude,
           "-I" + os.path.join(REF, "include"), "-I" + os.path.join(ROOT, "include"), PLUGIN]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "hl_codec_264_gfx950" not in r.stderr, r.stderr  # no warning from the plugin itself


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")), reason="reference sources are only in the build container")
def test_drop_in_driver_is_built():
    assert os.path.exists(DROP_IN), "make -C oracle ref builds oracle/_ref/drop_in_enc"
    syms = subprocess.run(["nm", DROP_IN], capture_output=True, text=True).stdout
    for s in ("hl_codec_264_gfx950_install", "hl_codec_encode", "hl_codec_264_plugin_def_t"):
        assert s in syms, s


CASES = ([c for c in GOLDEN_CONFIGS if c[0] in ("cif_ippp_qp31_me8", "qcif_gop3_qp20_me4", "w480_h272_qp28_me16")] + GOLDEN_ET_CONFIGS[:3] +
         [c for c in GOLDEN_RC_CONFIGS if c[0] in ("rc_qcif_100k_gop5", "rc_qcif_bu11_gop6", "rc_qcif_60k_qp20_36")] +
         [c for c in GOLDEN_MRF_CONFIGS if c[0] in ("mrf4_cif_qp31_nodb", "mrf8_cif_qp26", "mrf2_720p_qp28")])


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", CASES, ids=[c[0] for c in CASES])
def test_drop_in_through_hl_codec_encode(gpu, cfg):
    if not os.path.exists(DROP_IN):
        pytest.fail("oracle/_ref/drop_in_enc missing (built in the build container by make -C oracle ref)")
    name, w, h, n, qp, mer, db, gop, seed = cfg[:9]
    et = -1 if GOLD[name].get("early_term", 0) else 0  # -1: leave the hl_codec_create default (1)
    env = dict(os.environ)
    if cfg in GOLDEN_RC_CONFIGS:  # rc_bitrate etc. on the hl_codec_t (oracle/drop_in_harness.c)
        env.update(HL_REF_RC_BITRATE=str(cfg[9]), HL_REF_RC_BASICUNIT=str(cfg[10]), HL_REF_RC_QP_MIN=str(cfg[11]),
                   HL_REF_RC_QP_MAX=str(cfg[12]))
    if cfg in GOLDEN_MRF_CONFIGS:  # hl_codec_t.max_ref_frame, forwarded by the plugin
        env.update(HL_REF_MAX_REF_FRAME=str(cfg[9]))
    with tempfile.TemporaryDirectory() as td:
        inp, out = os.path.join(td, "in.yuv"), os.path.join(td, "out.264")
        golden_input(cfg).tofile(inp)
        r = subprocess.run([DROP_IN, str(w), str(h), str(n), str(qp), str(mer), str(db), str(gop), str(et), inp, out],
                           capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr
        got = open(out, "rb").read()
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    assert got == ref, f"{name}: first differing byte {first_diff(got, ref)}"


@pytest.mark.gpu
@pytest.mark.parametrize("lookahead", [4, 7])
@pytest.mark.parametrize("cfg", CASES[:2] + [c for c in CASES if c in GOLDEN_RC_CONFIGS][:1], ids=lambda c: c[0] if isinstance(c, tuple) else None)
def test_drop_in_lookahead(gpu, cfg, lookahead):
    # the plugin's opt-in look-ahead (HL_AMD_LOOKAHEAD): hl_codec_encode hands
    # out each frame's bytes lookahead - 1 calls late and the harness drains
    # the rest with hl_codec_264_gfx950_flush -- the same stream, including
    # frame counts that are not multiples of the look-ahead
    if not os.path.exists(DROP_IN):
        pytest.fail("oracle/_ref/drop_in_enc missing (built in the build container by make -C oracle ref)")
    name, w, h, n, qp, mer, db, gop, seed = cfg[:9]
    et = -1 if GOLD[name].get("early_term", 0) else 0
    env = dict(os.environ, HL_AMD_LOOKAHEAD=str(lookahead))
    if cfg in GOLDEN_RC_CONFIGS:
        env.update(HL_REF_RC_BITRATE=str(cfg[9]), HL_REF_RC_BASICUNIT=str(cfg[10]), HL_REF_RC_QP_MIN=str(cfg[11]),
                   HL_REF_RC_QP_MAX=str(cfg[12]))
    with tempfile.TemporaryDirectory() as td:
        inp, out = os.path.join(td, "in.yuv"), os.path.join(td, "out.264")
        golden_input(cfg).tofile(inp)
        r = subprocess.run([DROP_IN, str(w), str(h), str(n), str(qp), str(mer), str(db), str(gop), str(et), inp, out],
                           capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr
        got = open(out, "rb").read()
    ref = open(os.path.join(GOLDEN, name + ".264"), "rb").read()
    assert got == ref, f"{name} (look-ahead {lookahead}): first differing byte {first_diff(got, ref)}"


SVC_GOLD = json.load(open(os.path.join(GOLDEN, "svc_golden.json")))


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(SVC_GOLD) + ["svc2_qcif_qp28_db+lookahead"])
def test_drop_in_svc_through_hl_codec_encode(gpu, name):
    """Spatial SVC through the reference's own API with the gfx950 plugin:
    hl_codec_add_layer per layer, then hl_codec_encode per layer per frame
    (oracle/drop_in_harness.c svc mode), every access unit equal to the
    reference encoder's (tests/golden/svc_golden.json).  "+lookahead": with
    HL_AMD_LOOKAHEAD set, which an encoder with layers ignores."""
    import hashlib

    from hartallo_amd import synth

    if not os.path.exists(DROP_IN):
        pytest.fail("oracle/_ref/drop_in_enc missing (built in the build container by make -C oracle ref)")
    env = dict(os.environ)
    if name.endswith("+lookahead"):
        name = name[:-len("+lookahead")]
        env["HL_AMD_LOOKAHEAD"] = "4"
    g = SVC_GOLD[name]
    L, w0, h0, n = g["layers"], g["w0"], g["h0"], g["frames"]
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, n, g["seed"])
    et = -1 if g["early_term"] else 0
    with tempfile.TemporaryDirectory() as td:
        ins = []
        for l in range(L):
            ins.append(os.path.join(td, f"in{l}.yuv"))
            clips[l][:n].tofile(ins[-1])
        pre = os.path.join(td, "out")
        r = subprocess.run([DROP_IN, "svc", str(L), str(w0), str(h0), str(n), str(g["qp"]), str(g["me_range"]), str(g["deblock"]),
                            str(g["gop"]), str(et), pre] + ins, capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0, r.stderr
        got = open(pre + ".264", "rb").read()
        idx = [0] + [int(x) for x in open(pre + ".idx").read().split()]
    aus = [got[idx[i]:idx[i + 1]] for i in range(len(idx) - 1)]
    assert len(aus) == n
    for i, au in enumerate(aus):
        assert hashlib.md5(au).hexdigest() == g["au_md5"][i], f"{name}: access unit {i} differs ({len(au)} vs {g['au_bytes'][i]} bytes)"


# The reference decoder reads MbToSliceGroupMap uninitialised: it is
# realloc'd per slice header (hl_codec_264_slice.c:83) and never filled for
# one slice group, and NextMbAddress (slice.c:1660) compares its entries, so
# decoding works only when those words happen to be equal, as they are in
# fresh pages (MemorySanitizer: use-of-uninitialized-value at slice.c:1660,
# origin slice.c:83).  Whether they are depends on the process's heap
# history: one more codec object allocated before the decoder's first slice
# header is enough to make the stock decoder lose macroblocks.  The decode
# tests therefore run with glibc's MALLOC_PERTURB_, which fills every
# allocation with one byte value -- the condition the reference decoder
# silently relies on -- for the stock decoder and the drop-in alike.
DEC_ENV = dict(os.environ, MALLOC_PERTURB_="85")
DECODABLE = [c for c in GOLDEN_CONFIGS + GOLDEN_ET_CONFIGS + GOLDEN_RC_CONFIGS if "decoded_md5" in GOLD[c[0]]]


def _decode(tool, stream_path, out_path, *extra):
    r = subprocess.run([tool, *extra, stream_path, out_path], capture_output=True, text=True, timeout=240, env=DEC_ENV)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.skipif(not os.path.exists(DROP_IN_DEC), reason="oracle/_ref/drop_in_dec not built (make -C oracle ref)")
@pytest.mark.parametrize("cfg", DECODABLE, ids=[c[0] for c in DECODABLE])
def test_decode_after_install(cfg, tmp_path):
    """hl_codec_decode on a codec created after hl_codec_264_gfx950_install
    (the stock H.264 plugin is then out of the registry, hl_codec.c:182-229):
    the plugin's decode slot forwards to a stock codec it owns and returns
    exactly the pictures the reference decoder makes (decoded_md5,
    tests/golden/make_decoded_golden.py); encoding on that object afterwards is
    refused as the stock plugin refuses it (hl_codec_264.c:447-452).  CPU
    only: decoding never reaches the GPU library."""
    import hashlib

    import numpy as np

    name, w, h = cfg[0], cfg[1], cfg[2]
    info = _decode(DROP_IN_DEC, os.path.join(GOLDEN, name + ".264"), str(tmp_path / "d.yuv"), "dec")
    assert info["plugin_is_gfx950"] == 1 and info["errors"] == 0, info
    assert info["encode_after_decode"] == info["invalid_operation"], info
    d = np.fromfile(tmp_path / "d.yuv", np.uint8).reshape(-1, w * h * 3 // 2)
    assert [hashlib.md5(p.tobytes()).hexdigest() for p in d] == GOLD[name]["decoded_md5"]


@pytest.mark.skipif(not (os.path.exists(DROP_IN_DEC) and os.path.exists(REF_DEC)), reason="oracle/_ref decoders not built")
@pytest.mark.parametrize("cfg", GOLDEN_MRF_CONFIGS, ids=[c[0] for c in GOLDEN_MRF_CONFIGS])
def test_decode_after_install_max_ref_frame(cfg, tmp_path):
    """The max_ref_frame goldens (several reference frames in the SPS) decode
    through the installed plugin to the stock decoder's pictures."""
    name = cfg[0]
    stream = os.path.join(GOLDEN, name + ".264")
    a = _decode(DROP_IN_DEC, stream, str(tmp_path / "a.yuv"), "dec")
    b = _decode(REF_DEC, stream, str(tmp_path / "b.yuv"))
    assert a["errors"] == 0 and b["errors"] == 0 and a["frames"] == b["frames"] == cfg[3], (a, b)
    assert (tmp_path / "a.yuv").read_bytes() == (tmp_path / "b.yuv").read_bytes()
