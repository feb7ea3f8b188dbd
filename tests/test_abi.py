"""The drop-in boundary: the C-ABI library loads, exports every symbol
include/hartallo_amd.h declares, and fails loudly (no CPU fallback) when no
GPU is present.  No compute calls are made here."""
import ctypes
import os
import re

import pytest

from hl_testlib import ROOT

HEADER = os.path.join(ROOT, "include", "hartallo_amd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hl_amd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("hl_amd_encoder_create", "hl_amd_encode", "hl_amd_encode_device", "hl_amd_encoder_destroy"):
        assert must in names


def test_library_exports_every_declared_symbol():
    import hartallo_amd

    lib = hartallo_amd.load_library()
    assert os.path.samefile(hartallo_amd.LIB_PATH, os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so"))
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(hartallo_amd.EXPORTED_SYMBOLS)
    assert b"gfx950" in lib.hl_amd_version()


def test_library_is_a_gfx950_code_object():
    blob = open(os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so"), "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import hartallo_amd

    with pytest.raises(hartallo_amd.HlAmdError) as e:
        hartallo_amd.Encoder(352, 288)
    assert e.value.code != 0


def test_parameter_validation_before_device():
    import hartallo_amd
    from hartallo_amd._lib import _Params

    lib = hartallo_amd.load_library()
    h = ctypes.c_void_p()
    for bad in ((1920, 1080, 28), (0, 16, 28), (352, 288, 52)):
        p = _Params(bad[0], bad[1], bad[2], 16, 1, 30, 0, 0)
        rc = lib.hl_amd_encoder_create(ctypes.byref(p), ctypes.byref(h))
        assert rc in (1, 4), bad
    p = _Params(32, 16, 28, 16, 1, 30, 1, 0)  # early termination needs W, H >= 32 (rdo.c:895-896)
    assert lib.hl_amd_encoder_create(ctypes.byref(p), ctypes.byref(h)) == 4
