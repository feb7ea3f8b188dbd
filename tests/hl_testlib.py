"""Test support: ctypes bindings of the CPU oracle (oracle/_build/
libhloracle.so), of the host emulation of the kernel logic (tests/emu/
libhl_emu.so) and shared helpers.  TEST INFRASTRUCTURE ONLY -- the product
(hartallo_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from hartallo_amd import synth  # noqa: E402

ORACLE_LIB = os.path.join(ROOT, "oracle", "_build", "libhloracle.so")
EMU_LIB = os.environ.get("HL_EMU_LIB") or os.path.join(ROOT, "tests", "emu", "libhl_emu.so")  # HL_EMU_LIB: the sanitizer build (tests/test_sanitizers.py)
REF_ENC = os.path.join(ROOT, "oracle", "_ref", "ref_enc")
GOLDEN = os.path.join(ROOT, "tests", "golden")


class _OParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("width", "height", "qp", "me_range", "deblock", "gop_size", "early_term")]


_oracle = None
_emu = None


def oracle_lib():
    global _oracle
    if _oracle is None:
        lib = ctypes.CDLL(ORACLE_LIB)
        lib.hlo_create.argtypes = [ctypes.POINTER(_OParams)]
        lib.hlo_create.restype = ctypes.c_void_p
        lib.hlo_destroy.argtypes = [ctypes.c_void_p]
        lib.hlo_encode_frame.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        lib.hlo_encode_frame.restype = ctypes.c_int
        lib.hlo_recon.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.hlo_recon.restype = ctypes.c_void_p
        lib.hlo_rdo_overflows.argtypes = [ctypes.c_void_p]
        lib.hlo_rdo_overflows.restype = ctypes.c_int64
        lib.hlo_set_max_ref_frame.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _oracle = lib
    return _oracle


def emu_lib():
    global _emu
    if _emu is None:
        lib = ctypes.CDLL(EMU_LIB)
        lib.emu_create.restype = ctypes.c_void_p
        lib.emu_create.argtypes = [ctypes.c_int] * 7
        lib.emu_destroy.argtypes = [ctypes.c_void_p]
        lib.emu_encode_frame.restype = ctypes.c_long
        lib.emu_encode_frame.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_long]
        lib.emu_recon.restype = ctypes.c_void_p
        lib.emu_recon.argtypes = [ctypes.c_void_p, ctypes.c_int]
        lib.emu_set_rc.argtypes = [ctypes.c_void_p, ctypes.c_longlong] + [ctypes.c_int] * 5
        lib.emu_last_qp.argtypes = [ctypes.c_void_p]
        lib.emu_set_max_ref_frame.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _emu = lib
    return _emu


def _planes(frame: np.ndarray, w: int, h: int):
    n = w * h
    return frame[:n], frame[n:n + n // 4], frame[n + n // 4:n * 3 // 2]


def _recon(ptr_fn, w: int, h: int) -> np.ndarray:
    n = w * h
    parts = []
    for p, sz in ((0, n), (1, n // 4), (2, n // 4)):
        parts.append(np.ctypeslib.as_array(ctypes.cast(ptr_fn(p), ctypes.POINTER(ctypes.c_uint8)), shape=(sz,)).copy())
    return np.concatenate(parts)


class OracleEncoder:
    """CPU restatement of the reference encoder (oracle/hl_oracle.c)."""

    def __init__(self, w, h, qp=28, me_range=16, deblock=1, gop=30, early_term=0, max_ref_frame=1):
        self.lib = oracle_lib()
        self.w, self.h = w, h
        p = _OParams(w, h, qp, me_range, deblock, gop, early_term)
        self.h_ = self.lib.hlo_create(ctypes.byref(p))
        if not self.h_:
            raise ValueError("oracle rejected parameters")
        if max_ref_frame != 1:
            assert self.lib.hlo_set_max_ref_frame(ctypes.c_void_p(self.h_), max_ref_frame) == 0
        self.out = np.zeros(w * h * 4 + (1 << 20), np.uint8)

    def encode(self, frame: np.ndarray) -> bytes:
        y, u, v = _planes(frame, self.w, self.h)
        n = ctypes.c_size_t()
        rc = self.lib.hlo_encode_frame(ctypes.c_void_p(self.h_), y.ctypes.data, u.ctypes.data, v.ctypes.data, self.out.ctypes.data,
                                       self.out.size, ctypes.byref(n))
        assert rc == 0
        return self.out[:n.value].tobytes()

    def recon(self) -> np.ndarray:
        return _recon(lambda p: self.lib.hlo_recon(ctypes.c_void_p(self.h_), p), self.w, self.h)

    def rdo_overflows(self) -> int:
        return self.lib.hlo_rdo_overflows(ctypes.c_void_p(self.h_))

    def __del__(self):
        if getattr(self, "h_", None):
            self.lib.hlo_destroy(ctypes.c_void_p(self.h_))


class EmuEncoder:
    """Host build of the gfx950 kernel logic (tests/emu/hl_emu.hip)."""

    def __init__(self, w, h, qp=28, me_range=16, deblock=1, gop=30, early_term=0, max_ref_frame=1):
        self.lib = emu_lib()
        self.w, self.h = w, h
        self.h_ = self.lib.emu_create(w, h, qp, me_range, deblock, gop, early_term)
        if max_ref_frame != 1:
            self.lib.emu_set_max_ref_frame(ctypes.c_void_p(self.h_), max_ref_frame)
        self.out = np.zeros(w * h * 4 + (1 << 20), np.uint8)

    def set_rate_control(self, bitrate, fps_num=1, fps_den=15, basicunit=-1, qp_min=-1, qp_max=-1):
        assert self.lib.emu_set_rc(ctypes.c_void_p(self.h_), bitrate, fps_num, fps_den, basicunit, qp_min, qp_max) == 0

    def last_qp(self) -> int:
        return self.lib.emu_last_qp(ctypes.c_void_p(self.h_))

    def encode(self, frame: np.ndarray) -> bytes:
        y, u, v = _planes(frame, self.w, self.h)
        n = self.lib.emu_encode_frame(ctypes.c_void_p(self.h_), y.ctypes.data, u.ctypes.data, v.ctypes.data, self.out.ctypes.data,
                                      self.out.size)
        assert n > 0
        return self.out[:n].tobytes()

    def recon(self) -> np.ndarray:
        return _recon(lambda p: self.lib.emu_recon(ctypes.c_void_p(self.h_), p), self.w, self.h)

    def __del__(self):
        if getattr(self, "h_", None):
            self.lib.emu_destroy(ctypes.c_void_p(self.h_))


class EmuSvcEncoder:
    """Spatial SVC through the host build of the kernel logic: layer l is
    (w0 << l) x (h0 << l); encode(layer, frame) returns what the reference
    SVC harness writes for that call (oracle/ref_svc_harness.c)."""

    def __init__(self, w0, h0, layers, qp=28, me_range=16, deblock=1, gop=30, early_term=0):
        lib = emu_lib()
        if not hasattr(lib, "_svc_bound"):
            lib.emu_svc_create.restype = ctypes.c_void_p
            lib.emu_svc_create.argtypes = [ctypes.c_int] * 8
            lib.emu_svc_destroy.argtypes = [ctypes.c_void_p]
            lib.emu_svc_encode.restype = ctypes.c_long
            lib.emu_svc_encode.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_long]
            lib.emu_svc_recon.restype = ctypes.c_void_p
            lib.emu_svc_recon.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            lib.emu_svc_unpinned.argtypes = [ctypes.c_void_p]
            lib.emu_svc_set_range.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
            lib.emu_svc_layer_state_bytes.restype = ctypes.c_long
            lib.emu_svc_layer_state_bytes.argtypes = [ctypes.c_void_p, ctypes.c_int]
            lib.emu_svc_export.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            lib.emu_svc_import.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
            lib.emu_svc_last_hdr.restype = ctypes.c_long
            lib.emu_svc_last_hdr.argtypes = [ctypes.c_void_p]
            lib._svc_bound = True
        self.lib = lib
        self.w0, self.h0, self.L = w0, h0, layers
        self.h_ = lib.emu_svc_create(w0, h0, layers, qp, me_range, deblock, gop, early_term)
        assert self.h_
        w, h = w0 << (layers - 1), h0 << (layers - 1)
        self.out = np.zeros(w * h * 3 * layers + (1 << 20), np.uint8)

    def encode(self, layer: int, frame: np.ndarray) -> bytes:
        w, h = self.w0 << layer, self.h0 << layer
        y, u, v = _planes(frame, w, h)
        n = self.lib.emu_svc_encode(ctypes.c_void_p(self.h_), layer, y.ctypes.data, u.ctypes.data, v.ctypes.data, self.out.ctypes.data,
                                    self.out.size)
        assert n >= 0, n
        return self.out[:n].tobytes()

    def recon(self, layer: int) -> np.ndarray:
        w, h = self.w0 << layer, self.h0 << layer
        return _recon(lambda p: self.lib.emu_svc_recon(ctypes.c_void_p(self.h_), layer, p), w, h)

    def unpinned(self) -> int:
        return self.lib.emu_svc_unpinned(ctypes.c_void_p(self.h_))

    def last_hdr(self) -> int:
        """header bytes at the start of the last encode() output"""
        return self.lib.emu_svc_last_hdr(ctypes.c_void_p(self.h_))

    def set_range(self, first: int, last: int):
        assert self.lib.emu_svc_set_range(ctypes.c_void_p(self.h_), first, last) == 0

    def layer_state_bytes(self, layer: int) -> int:
        return self.lib.emu_svc_layer_state_bytes(ctypes.c_void_p(self.h_), layer)

    def export_layer(self, layer: int) -> np.ndarray:
        buf = np.zeros(self.layer_state_bytes(layer), np.uint8)
        assert self.lib.emu_svc_export(ctypes.c_void_p(self.h_), layer, buf.ctypes.data) == 0
        return buf

    def import_layer(self, layer: int, buf: np.ndarray):
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        assert self.lib.emu_svc_import(ctypes.c_void_p(self.h_), layer, buf.ctypes.data) == 0

    def __del__(self):
        if getattr(self, "h_", None):
            self.lib.emu_svc_destroy(ctypes.c_void_p(self.h_))


class GpuEncoder:
    """The product (libhartallo_amd.so) with the same encode() shape."""

    def __init__(self, w, h, qp=28, me_range=16, deblock=1, gop=30, early_term=0, max_ref_frame=1):
        from hartallo_amd import Encoder

        self.enc = Encoder(w, h, qp, me_range, deblock, gop, early_term)
        if max_ref_frame != 1:
            self.enc.set_max_ref_frame(max_ref_frame)
        self.w, self.h = w, h

    def encode(self, frame: np.ndarray) -> bytes:
        y, u, v = _planes(frame, self.w, self.h)
        return self.enc.encode(y, u, v).annexb()

    def recon(self) -> np.ndarray:
        return np.concatenate(self.enc.recon())

    def set_rate_control(self, *a, **k):
        self.enc.set_rate_control(*a, **k)

    def last_qp(self) -> int:
        return self.enc.last_qp()


def significant_records(r: np.ndarray) -> np.ndarray:
    """Copy of an MbRecord array with the fields the slice writer does not
    read for that macroblock zeroed (they hold LDS scratch of the search,
    which is not part of the result): mv of intra MBs, levels of uncoded
    blocks, I16 / I4 / chroma syntax of MBs without it, padding."""
    r = r.copy()
    if "dbg" in r.dtype.names:
        r["dbg"] = 0
    intra = (r["flags"] & 1) != 0
    skip = (r["flags"] & 4) != 0
    r["pad0"] = 0
    # motion of the partitions the MB has (P_Skip: [0][0]); none for intra
    pi = np.arange(4)[None, :, None]
    spi = np.arange(4)[None, None, :]
    num_part = np.where(intra, 0, np.maximum(r["num_part"], 1))[:, None, None]
    num_sub = np.where(r["flags"][:, None] & 4, 1, np.maximum(r["num_sub"], 1))[:, :, None]
    keep = (pi < num_part) & (spi < num_sub)
    r["mv"][~keep] = 0
    for f in ("num_sub", "sub_mb_type", "mvd"):
        r[f][intra | skip] = 0
    r["i16dc"][r["pm0"] != 3] = 0
    r["nc_dc"][r["pm0"] != 3] = 0
    for f in ("i4mode", "prev_flag", "rem_mode"):
        r[f][r["pm0"] != 2] = 0
    for f in ("chroma_mode", "i16mode"):
        r[f][~intra] = 0
    coded8 = (r["cbp_l"][:, None] >> (np.arange(16)[None, :] >> 2)) & 1
    r["luma"][coded8 == 0] = 0
    r["nc_luma"][coded8 == 0] = 0
    r["cdc"][(r["cbp_c"] & 3) == 0] = 0
    r["cac"][(r["cbp_c"] & 2) == 0] = 0
    r["nc_cac"][(r["cbp_c"] & 2) == 0] = 0
    return r


def first_record_diff(recs_a, recs_b, mbw: int) -> str:
    """First (picture, MB, field) where two lists of per-picture MbRecord
    arrays (Encoder.debug_records) differ in a field the writer reads, as a
    message for a failing parity assertion."""
    for f, (a, b) in enumerate(zip(recs_a, recs_b)):
        if a is None or b is None:
            return f"picture {f}: records not kept"
        if "dbg" in a.dtype.names:  # diagnostic build: the first MB whose inputs differ, in decision order
            order = sorted(range(len(a)), key=lambda m: ((m % mbw) + 2 * (m // mbw), m // mbw))
            for m in order:
                if not np.array_equal(a[m]["dbg"], b[m]["dbg"]):
                    k = int(np.nonzero(a[m]["dbg"] != b[m]["dbg"])[0][0])
                    names = ["top", "left", "chroma nb", "nb state/motion", "nC/ext", "live tc/cbp", "cac/src", "chain"]
                    print(f"  picture {f}: first input difference at MB {m} ({m % mbw},{m // mbw}) in {names[k]}: "
                          f"{a[m]['dbg'].tolist()} vs {b[m]['dbg'].tolist()}", flush=True)
                    break
        a, b = significant_records(a), significant_records(b)
        if a.tobytes() == b.tobytes():
            continue
        for m in range(len(a)):
            if a[m].tobytes() != b[m].tobytes():
                for name in a.dtype.names:
                    if not np.array_equal(a[m][name], b[m][name]):
                        va, vb = np.asarray(a[m][name]).ravel(), np.asarray(b[m][name]).ravel()
                        i = int(np.nonzero(va != vb)[0][0])
                        return (f"picture {f} MB {m} ({m % mbw},{m // mbw}) e_type {a[m]['e_type']}/{b[m]['e_type']} field {name}[{i}:]: "
                                f"{va[i:i + 16].tolist()} vs {vb[i:i + 16].tolist()}")
    return "records equal (difference after the decisions: writer or deblocking)"


def md5(b) -> str:
    return hashlib.md5(bytes(b)).hexdigest()


def first_diff(a: bytes, b: bytes) -> int:
    for i in range(min(len(a), len(b))):
        if a[i] != b[i]:
            return i
    return -1 if len(a) == len(b) else min(len(a), len(b))


# Golden configurations: (name, W, H, frames, qp, me_range, deblock, gop, seed).
# tests/golden/make_golden.py encodes them with the reference (oracle/_ref/ref_enc).
GOLDEN_CONFIGS = [
    ("cif_i_qp31", 352, 288, 1, 31, 8, 0, 400, 1),           # config 1: test_encoder.c settings
    ("cif_ippp_qp31_me8", 352, 288, 6, 31, 8, 0, 400, 2),
    ("qcif_ippp_qp28_db", 176, 144, 8, 28, 16, 1, 30, 3),
    ("qcif_gop3_qp20_me4", 176, 144, 8, 20, 4, 1, 3, 4),
    ("qcif_qp40_me16_gop4", 176, 144, 8, 40, 16, 1, 4, 5),
    ("qcif_qp12_me2", 176, 144, 4, 12, 2, 1, 400, 6),
    ("qcif_qp51", 176, 144, 4, 51, 8, 1, 400, 7),
    ("tiny_32x16_qp26", 32, 16, 6, 26, 8, 1, 2, 8),
    ("qcif_qp0_me1", 176, 144, 3, 0, 1, 1, 400, 9),
    ("w480_h272_qp28_me16", 480, 272, 4, 28, 16, 1, 30, 10),
    # below QP 10 the reference's lambda shift count is negative (slice.c:1766,
    # hl_prims.h rdo_lambda): QP 4 -> 2^30.  (QP 7-9 give INT_MIN, a negative
    # lambda: the reference's own encode then fails, tests/test_drop_in.py.)
    ("qcif_qp4_me4", 176, 144, 3, 4, 4, 1, 400, 11),
]

# Configurations whose encode the reference itself FAILS: at QP 7-9 its
# lambda is negative (rdo_lambda), the RDO picks the costliest candidates,
# and the first P picture's slice outgrows the (mb_count << 8) + 4096 slice
# buffer (encode.c:192) -> HL_ERROR_TOOSHORT (15) from the escape
# (rbsp.c:617-620).  golden.json keeps the frames before the failure, the
# failing frame and the error; every implementation must fail there too.
GOLDEN_FAIL_CONFIGS = [
    ("fail_qcif_qp8_neg_lambda", 176, 144, 4, 8, 8, 1, 400, 12),
]


# Early-termination goldens (me_early_term_flag = 1, the hl_codec_create
# default, hl_types.h:67): same layout, encoded by make_golden.py with
# early_term 1.  Early termination needs W, H >= 32 (rdo.c:895-896 read one
# sample around the MB quadrants).
GOLDEN_ET_CONFIGS = [
    ("et_qcif_ippp_qp28", 176, 144, 6, 28, 16, 1, 30, 41),
    ("et_cif_qp31_me8", 352, 288, 5, 31, 8, 0, 400, 42),
    ("et_w480_qp20_gop3", 480, 272, 5, 20, 16, 1, 3, 43),
    ("et_w64_h32_qp36", 64, 32, 6, 36, 4, 1, 4, 44),
    ("et_qcif_qp12_me2", 176, 144, 4, 12, 2, 1, 400, 45),
]


# Rate-control goldens (hl_codec_t.rc_bitrate > 0, hl_codec_264.c:719-742):
# (name, W, H, frames, qp, me_range, deblock, gop, seed, bitrate, basicunit,
# qp_min, qp_max), fps 1/15 as test_encoder.c sets it.  Several GOPs each, so
# the model's GOP-to-GOP QP carry (rc.c:844-882) is exercised; bu11 runs the
# basic-unit bookkeeping.
GOLDEN_RC_CONFIGS = [
    ("rc_qcif_100k_gop5", 176, 144, 16, 28, 8, 1, 5, 51, 100000, -1, -1, -1),
    ("rc_qcif_30k_gop6", 176, 144, 14, 28, 8, 1, 6, 52, 30000, -1, -1, -1),
    ("rc_qcif_bu11_gop6", 176, 144, 13, 28, 8, 1, 6, 53, 100000, 11, -1, -1),
    ("rc_cif_200k_gop4_nodb", 352, 288, 9, 28, 8, 0, 4, 54, 200000, -1, -1, -1),
    ("rc_qcif_1m5_gop6", 176, 144, 13, 28, 16, 1, 6, 55, 1500000, -1, -1, -1),
    ("rc_qcif_60k_qp20_36", 176, 144, 12, 28, 8, 1, 5, 56, 60000, -1, 20, 36),
]


# max_ref_frame goldens (hl_codec_t.max_ref_frame > 1, the SPS's
# max_num_ref_frames = min(MaxDpbMbs / PicSizeInMbs, max_ref_frame) and the
# PPS's num_ref_idx_l0_default_active_minus1, hl_codec_264_sps.c:620-636,
# hl_codec_264_pps.c:291): (name, W, H, frames, qp, me_range, deblock, gop,
# seed, max_ref_frame).  CIF allows 6 reference frames at its level 1.3
# (2376 / 396), so 8 is clipped; 720p allows 5 (18000 / 3600).
GOLDEN_MRF_CONFIGS = [
    ("mrf2_cif_qp28_gop3", 352, 288, 5, 28, 8, 1, 3, 61, 2),
    ("mrf4_cif_qp31_nodb", 352, 288, 4, 31, 8, 0, 30, 62, 4),
    ("mrf8_cif_qp26", 352, 288, 3, 26, 16, 1, 400, 63, 8),
    ("mrf2_720p_qp28", 1280, 720, 3, 28, 16, 1, 30, 64, 2),
    ("mrf4_720p_qp32", 1280, 720, 3, 32, 16, 1, 30, 65, 4),
    # above 16: the reference writes min(MaxDpbMbs / PicSizeInMbs, max_ref_frame) (sps.c:635-636)
    ("mrf32_720p_qp30", 1280, 720, 2, 30, 8, 1, 30, 66, 32),
    ("mrf17_cif_qp30", 352, 288, 3, 30, 8, 1, 30, 67, 17),
]


def slice_qps(stream: bytes, pic_init_qp: int) -> list:
    """SliceQPY of every slice NAL of an Annex-B stream (slice_qp_delta of the
    Baseline slice header this encoder writes, slice.c:660-900)."""
    out, i = [], 0
    while True:
        j = stream.find(b"\x00\x00\x01", i)
        if j < 0:
            return out
        i = j + 3
        t = stream[i] & 31
        if t not in (1, 5):
            continue
        bits = "".join(f"{b:08b}" for b in stream[i + 1:i + 24])
        pos = [0]

        def u(n):
            v = int(bits[pos[0]:pos[0] + n], 2)
            pos[0] += n
            return v

        def ue():
            z = 0
            while bits[pos[0]] == "0":
                z += 1
                pos[0] += 1
            pos[0] += 1
            return (1 << z) - 1 + (u(z) if z else 0)

        ue(), ue(), ue(), u(8)          # first_mb, slice_type, pps id, frame_num
        if t == 5:
            ue(), u(1), u(1)            # idr_pic_id, dec_ref_pic_marking
        else:
            u(1), ue(), u(1), u(1)      # override, num_ref_idx, modification, marking
        k = ue()
        out.append(pic_init_qp + ((k + 1) // 2 if k & 1 else -(k // 2)))


def check_reference_failure(name, make_encoder, encode_ok, gold):
    """A GOLDEN_FAIL_CONFIGS entry: the frames before the reference's failing
    frame byte for byte (stream and recon MD5s), then the failing frame
    refused.  encode_ok(enc, frame) -> bytes, or None when the
    implementation refused the frame."""
    cfg = next(c for c in GOLDEN_FAIL_CONFIGS if c[0] == name)
    g = gold[name]
    clip = golden_input(cfg)
    enc = make_encoder(cfg)
    out = b""
    for f in range(g["fail_frame"]):
        b = encode_ok(enc, clip[f])
        assert b is not None, f"{name}: frame {f} refused, the reference coded it"
        out += b
    assert md5(out) == g["stream_md5"], f"{name}: the frames before the failure differ from the reference's"
    assert encode_ok(enc, clip[g["fail_frame"]]) is None, f"{name}: frame {g['fail_frame']} coded, the reference failed it"


def golden_input(cfg) -> np.ndarray:
    _, w, h, n, _, _, _, _, seed = cfg[:9]
    return synth.clip(w, h, n, seed)
