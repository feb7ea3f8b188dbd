"""ctypes binding of libhartallo_amd.so (include/hartallo_amd.h).

The library is the HIP build for gfx950; there is no CPU fallback.  Loading
fails loudly when the library is missing, and encoding fails loudly when no
GPU is present.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libhartallo_amd.so")

# include/hartallo_amd.h
HL_AMD_SUCCESS = 0
HL_AMD_ERROR_INVALID_PARAMETER = 1
HL_AMD_ERROR_INVALID_STATE = 3
HL_AMD_ERROR_INVALID_FORMAT = 4
HL_AMD_ERROR_NOT_FOUND = 6
HL_AMD_ERROR_NOT_IMPLEMENTED = 7
HL_AMD_ERROR_OUTOFMEMMORY = 8
HL_AMD_ERROR_OUTOFCAPACITY = 10
HL_AMD_ERROR_SYSTEM = 13
HL_AMD_ERROR_TOOSHORT = 15
HL_AMD_RESULT_TYPE_DATA = 1
HL_AMD_RESULT_TYPE_HDR = 2

# every symbol include/hartallo_amd.h declares
EXPORTED_SYMBOLS = (
    "hl_amd_encoder_create",
    "hl_amd_encoder_destroy",
    "hl_amd_encode",
    "hl_amd_set_lookahead",
    "hl_amd_flush",
    "hl_amd_encode_device",
    "hl_amd_encode_batch",
    "hl_amd_encode_streams",
    "hl_amd_set_pipeline",
    "hl_amd_set_rate_control",
    "hl_amd_set_max_ref_frame",
    "hl_amd_last_qp",
    "hl_amd_pipeline_occupancy",
    "hl_amd_bench_planes",
    "hl_amd_get_recon",
    "hl_amd_set_timing",
    "hl_amd_get_timing",
    "hl_amd_last_reruns",
    "hl_amd_last_chain_walks",
    "hl_amd_last_mb_launches",
    "hl_amd_last_batch_stats",
    "hl_amd_set_intra_helpers",
    "hl_amd_last_helper_stats",
    "hl_amd_last_fam3_stats",
    "hl_amd_profile_counters",
    "hl_amd_debug_records",
    "hl_amd_record_size",
    "hl_amd_debug_chain",
    "hl_amd_debug_recon",
    "hl_amd_add_layer",
    "hl_amd_encode_layer",
    "hl_amd_get_layer_recon",
    "hl_amd_svc_unpinned",
    "hl_amd_set_layer_range",
    "hl_amd_layer_state_bytes",
    "hl_amd_export_layer",
    "hl_amd_import_layer",
    "hl_amd_svc_layer_ms",
    "hl_amd_encode_layers_batch",
    "hl_amd_version",
)


class HlAmdError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with HL_ERROR {code}")
        self.code = code


class _Params(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("width", "height", "qp", "me_range", "deblock", "gop_size", "me_early_term", "device")]


class _Result(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_int32),
        ("hdr", ctypes.c_void_p),
        ("hdr_size", ctypes.c_size_t),
        ("data", ctypes.c_void_p),
        ("data_size", ctypes.c_size_t),
    ]


def _mb_record_dtype():
    """numpy mirror of MbRecord (hartallo_amd/csrc/hl_types.h)."""
    import numpy as np

    return np.dtype([
        ("e_type", "<i4"), ("mb_type", "<i4"), ("flags", "<i4"), ("pm0", "<i4"),
        ("cbp", "<i4"), ("cbp_l", "<i4"), ("cbp_c", "<i4"), ("cbp_l4x4", "<i4"),
        ("cbp_cdc", "<i4", 2), ("cbp_cac", "<i4", 2), ("num_part", "<i4"), ("num_sub", "<i4", 4), ("sub_mb_type", "<i4", 4),
        ("chroma_mode", "<i4"), ("i16mode", "<i4"), ("mvd", "<i2", (4, 4, 2)), ("mv", "<i2", (4, 4, 2)),
        ("prev_flag", "i1", 16), ("rem_mode", "i1", 16), ("i4mode", "i1", 16), ("nc_luma", "i1", 16), ("nc_cac", "i1", (2, 4)),
        ("nc_dc", "i1"), ("pad0", "i1", 3), ("luma", "<i2", (16, 16)), ("i16dc", "<i2", 16), ("cdc", "<i2", (2, 4)),
        ("cac", "<i2", (2, 4, 16)), ("mad", "<i4"), ("pad1", "<i4"),
    ])


try:
    MB_RECORD = _mb_record_dtype()
except ImportError:  # numpy is optional for the plain ctypes binding
    MB_RECORD = None

_lib = None
LOADED_PATH = None  # the library file load_library loaded (bench.py stamps counters with its hash)


def code_sha256(path: str) -> str:
    """SHA-256 of a built library's code and constants: its .hip_fatbin (the
    gfx950 code objects), .text (the host code), .rodata and .data sections,
    in that order (a missing one counts as empty).  Two links of
    the same sources can lay out the ELF string tables differently (the whole
    file's hash then differs while every instruction is the same); counters
    recorded on one are valid for the other."""
    import hashlib
    import struct

    data = open(path, "rb").read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]

    def name(off):
        return data[stroff + off:data.index(b"\0", stroff + off)].decode()

    by = {name(sn): (o, sz) for sn, _, _, _, o, sz in secs}
    h = hashlib.sha256()
    for sec in (".hip_fatbin", ".text", ".rodata", ".data"):
        o, sz = by.get(sec, (0, 0))
        h.update(data[o:o + sz])
    return h.hexdigest()


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Loads the HIP library.  torch (if installed) is imported first so the
    process ends up with one HIP runtime (torch ships its own
    libamdhip64.so.7, which then also satisfies this library)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} is missing: build it with `make product` (hipcc --offload-arch=gfx950)")
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(path)
    global LOADED_PATH
    LOADED_PATH = os.path.abspath(path)
    vp, i32 = ctypes.c_void_p, ctypes.c_int32
    lib.hl_amd_encoder_create.argtypes = [ctypes.POINTER(_Params), ctypes.POINTER(vp)]
    lib.hl_amd_encoder_create.restype = i32
    lib.hl_amd_encoder_destroy.argtypes = [vp]
    lib.hl_amd_encoder_destroy.restype = None
    for f in (lib.hl_amd_encode, lib.hl_amd_encode_device):
        f.argtypes = [vp, vp, vp, vp, ctypes.POINTER(_Result)]
        f.restype = i32
    pp = ctypes.POINTER(ctypes.c_void_p)
    lib.hl_amd_encode_batch.argtypes = [vp, i32, pp, pp, pp, ctypes.POINTER(_Result)]
    lib.hl_amd_encode_batch.restype = i32
    if hasattr(lib, "hl_amd_encode_streams"):  # (absent from builds before round 4 loaded through HL_LIB)
        lib.hl_amd_encode_streams.argtypes = [ctypes.POINTER(vp), i32, i32, pp, pp, pp, ctypes.POINTER(_Result)]
        lib.hl_amd_encode_streams.restype = i32
    lib.hl_amd_set_pipeline.argtypes = [vp, i32, i32, i32]
    lib.hl_amd_set_pipeline.restype = i32
    lib.hl_amd_set_rate_control.argtypes = [vp, ctypes.c_int64, i32, i32, i32, i32, i32]
    lib.hl_amd_set_rate_control.restype = i32
    if hasattr(lib, "hl_amd_set_max_ref_frame"):  # (absent from builds before round 5 loaded through HL_LIB)
        lib.hl_amd_set_max_ref_frame.argtypes = [vp, i32]
        lib.hl_amd_set_max_ref_frame.restype = i32
    lib.hl_amd_last_qp.argtypes = [vp]
    lib.hl_amd_last_qp.restype = i32
    lib.hl_amd_pipeline_occupancy.argtypes = []
    lib.hl_amd_pipeline_occupancy.restype = i32
    lib.hl_amd_bench_planes.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_float)]
    lib.hl_amd_bench_planes.restype = i32
    lib.hl_amd_get_recon.argtypes = [vp, vp, vp, vp]
    lib.hl_amd_get_recon.restype = i32
    lib.hl_amd_set_timing.argtypes = [vp, i32]
    lib.hl_amd_set_timing.restype = i32
    lib.hl_amd_get_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    lib.hl_amd_get_timing.restype = i32
    lib.hl_amd_last_reruns.argtypes = [vp]
    lib.hl_amd_last_reruns.restype = i32
    lib.hl_amd_last_chain_walks.argtypes = [vp]
    lib.hl_amd_last_chain_walks.restype = i32
    lib.hl_amd_last_mb_launches.argtypes = [vp]
    lib.hl_amd_last_mb_launches.restype = i32
    lib.hl_amd_last_batch_stats.argtypes = [vp, ctypes.POINTER(i32)]
    lib.hl_amd_last_batch_stats.restype = i32
    for name, args in (("hl_amd_set_intra_helpers", [vp, i32]), ("hl_amd_last_helper_stats", [vp, ctypes.POINTER(i32)]),
                       ("hl_amd_last_fam3_stats", [vp, ctypes.POINTER(i32)]), ("hl_amd_set_lookahead", [vp, i32]),
                       ("hl_amd_flush", [vp, ctypes.POINTER(_Result)])):
        if hasattr(lib, name):  # (absent from builds before round 4 loaded through HL_LIB)
            getattr(lib, name).argtypes = args
            getattr(lib, name).restype = i32
    lib.hl_amd_profile_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_ulonglong), i32]
    lib.hl_amd_profile_counters.restype = i32
    # diagnostics entry points (absent from older builds loaded through HL_LIB)
    for name, args in (("hl_amd_debug_records", [vp, i32, vp, ctypes.c_size_t]), ("hl_amd_debug_chain", [vp, i32, vp, ctypes.c_size_t]),
                       ("hl_amd_debug_recon", [vp, i32, vp, vp, vp]), ("hl_amd_record_size", [])):
        if hasattr(lib, name):
            getattr(lib, name).argtypes = args
            getattr(lib, name).restype = i32
    lib.hl_amd_add_layer.argtypes = [vp, i32, i32]
    lib.hl_amd_add_layer.restype = i32
    lib.hl_amd_encode_layer.argtypes = [vp, i32, i32, vp, vp, vp, i32, ctypes.POINTER(_Result)]
    lib.hl_amd_encode_layer.restype = i32
    lib.hl_amd_get_layer_recon.argtypes = [vp, i32, vp, vp, vp]
    lib.hl_amd_get_layer_recon.restype = i32
    lib.hl_amd_svc_unpinned.argtypes = [vp]
    lib.hl_amd_svc_unpinned.restype = i32
    lib.hl_amd_set_layer_range.argtypes = [vp, i32, i32]
    lib.hl_amd_set_layer_range.restype = i32
    lib.hl_amd_layer_state_bytes.argtypes = [vp, i32]
    lib.hl_amd_layer_state_bytes.restype = ctypes.c_size_t
    lib.hl_amd_export_layer.argtypes = [vp, i32, vp]
    lib.hl_amd_export_layer.restype = i32
    lib.hl_amd_import_layer.argtypes = [vp, i32, vp]
    lib.hl_amd_import_layer.restype = i32
    lib.hl_amd_encode_layers_batch.argtypes = [vp, i32, i32, pp, ctypes.POINTER(_Result)]
    lib.hl_amd_encode_layers_batch.restype = i32
    lib.hl_amd_svc_layer_ms.argtypes = [vp]
    lib.hl_amd_svc_layer_ms.restype = ctypes.c_float
    lib.hl_amd_version.argtypes = []
    lib.hl_amd_version.restype = ctypes.c_char_p
    _lib = lib
    return lib


@dataclass
class EncodeResult:
    """hl_codec_result_t of one encode() call (hl_codec.h:152-168)."""

    type: int
    data: bytes
    hdr: bytes

    def annexb(self) -> bytes:
        """Bytes the reference's test harness writes for this frame
        (test_encoder.c:220-236): headers when signalled, then a start code
        and the slice NAL."""
        out = self.hdr if self.type & HL_AMD_RESULT_TYPE_HDR else b""
        return out + b"\x00\x00\x01" + self.data


class Encoder:
    """One H.264 encode stream on one GPU (one hl_codec_t, not reentrant)."""

    def __init__(self, width: int, height: int, qp: int = 28, me_range: int = 16, deblock: int = 1, gop_size: int = 30,
                 me_early_term: int = 0, device: int = 0):
        self.lib = load_library()
        self.width, self.height = width, height
        p = _Params(width, height, qp, me_range, deblock, gop_size, me_early_term, device)
        h = ctypes.c_void_p()
        rc = self.lib.hl_amd_encoder_create(ctypes.byref(p), ctypes.byref(h))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encoder_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self.lib.hl_amd_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _result(self, r: _Result) -> EncodeResult:
        data = ctypes.string_at(r.data, r.data_size) if r.type & HL_AMD_RESULT_TYPE_DATA else b""
        hdr = ctypes.string_at(r.hdr, r.hdr_size) if r.type & HL_AMD_RESULT_TYPE_HDR else b""
        return EncodeResult(r.type, data, hdr)

    def encode(self, y, u, v) -> EncodeResult:
        """Encodes planar YUV420 from host memory (numpy uint8 arrays)."""
        import numpy as np

        ys = [np.ascontiguousarray(p, dtype=np.uint8) for p in (y, u, v)]
        if ys[0].size != self.width * self.height or ys[1].size != self.width * self.height // 4 or ys[2].size != ys[1].size:
            raise HlAmdError(HL_AMD_ERROR_INVALID_FORMAT, "encode (plane sizes)")
        r = _Result()
        rc = self.lib.hl_amd_encode(self._h, ys[0].ctypes.data, ys[1].ctypes.data, ys[2].ctypes.data, ctypes.byref(r))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode")
        return self._result(r)

    def set_lookahead(self, frames: int) -> None:
        """Look-ahead for per-frame callers (hl_amd_set_lookahead): encode()
        queues frames and codes them `frames` at a time; each call returns the
        next coded result in order (type 0 while the queue fills), flush()
        the rest."""
        rc = self.lib.hl_amd_set_lookahead(self._h, frames)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_set_lookahead")

    def flush(self) -> EncodeResult:
        """Codes what the look-ahead still queues and returns the next
        result (type 0 once none is left)."""
        r = _Result()
        rc = self.lib.hl_amd_flush(self._h, ctypes.byref(r))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_flush")
        return self._result(r)

    def encode_device(self, y_ptr: int, u_ptr: int, v_ptr: int, collect: bool = True):
        """Encodes planes already resident in device memory (raw pointers)."""
        r = _Result()
        rc = self.lib.hl_amd_encode_device(self._h, ctypes.c_void_p(y_ptr), ctypes.c_void_p(u_ptr), ctypes.c_void_p(v_ptr), ctypes.byref(r))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_device")
        return self._result(r) if collect else r.data_size

    def encode_batch_device(self, ptrs, collect: bool = True):
        """Encodes consecutive frames already resident in device memory;
        ptrs = [(y_ptr, u_ptr, v_ptr), ...].  Runs of P pictures are
        frame-pipelined (hl_amd_encode_batch); returns one result per frame
        (or, with collect=False, the total bitstream bytes)."""
        n = len(ptrs)
        arr = [(ctypes.c_void_p * n)(*[p[i] for p in ptrs]) for i in range(3)]
        res = (_Result * n)()
        rc = self.lib.hl_amd_encode_batch(self._h, n, arr[0], arr[1], arr[2], res)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_batch")
        self._last_batch = res  # the results stay valid until the next encode call
        return [self._result(r) for r in res] if collect else sum(r.data_size for r in res)

    @staticmethod
    def encode_streams_device(encoders, ptrs, collect: bool = True):
        """hl_amd_encode_streams: frames of several streams in shared
        pipelined runs; encoders[s] codes ptrs[s] (each a list of (y, u, v)
        device pointers, the same length).  Returns per stream its results (or,
        with collect=False, its total bitstream bytes)."""
        S, n = len(encoders), len(ptrs[0])
        assert len(ptrs) == S and all(len(p) == n for p in ptrs)
        lib = encoders[0].lib
        hs = (ctypes.c_void_p * S)(*[e._h for e in encoders])
        flat = [f for p in ptrs for f in p]
        arr = [(ctypes.c_void_p * (S * n))(*[f[i] for f in flat]) for i in range(3)]
        res = (_Result * (S * n))()
        rc = lib.hl_amd_encode_streams(hs, S, n, arr[0], arr[1], arr[2], res)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_streams")
        out = []
        for s, e in enumerate(encoders):
            rs = res[s * n:(s + 1) * n]
            e._last_batch = rs
            out.append([e._result(r) for r in rs] if collect else sum(r.data_size for r in rs))
        return out

    def last_batch_results(self):
        """The results of the last encode_batch_device call (also after
        collect=False), valid until the next encode call."""
        return [self._result(r) for r in self._last_batch]

    def set_rate_control(self, bitrate: int, fps_num: int = 1, fps_den: int = 15, basicunit: int = -1, qp_min: int = -1,
                         qp_max: int = -1):
        """Rate control (hl_codec_t.rc_bitrate > 0 and its companions; call
        before the first frame; bitrate <= 0 turns it off)."""
        rc = self.lib.hl_amd_set_rate_control(self._h, bitrate, fps_num, fps_den, basicunit, qp_min, qp_max)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_set_rate_control")

    def set_max_ref_frame(self, max_ref_frame: int):
        """hl_codec_t.max_ref_frame: SPS/PPS fields only (hl_codec_264_sps.c:620-636); before the first frame."""
        rc = self.lib.hl_amd_set_max_ref_frame(self._h, max_ref_frame)
        if rc:
            raise HlAmdError(rc, "hl_amd_set_max_ref_frame")

    def last_qp(self) -> int:
        """SliceQPY of the last encoded picture."""
        return self.lib.hl_amd_last_qp(self._h)

    def bench_planes(self, iters: int = 50) -> float:
        """average ms per launch of the quarter-pel plane kernel (diagnostics)"""
        ms = ctypes.c_float()
        rc = self.lib.hl_amd_bench_planes(self._h, iters, ctypes.byref(ms))
        if rc:
            raise HlAmdError(rc, "hl_amd_bench_planes")
        return ms.value

    def set_pipeline(self, workgroups: int, reach: int, window: int):
        rc = self.lib.hl_amd_set_pipeline(self._h, workgroups, reach, window)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_set_pipeline")

    def recon(self):
        import numpy as np

        y = np.empty(self.width * self.height, np.uint8)
        u = np.empty(self.width * self.height // 4, np.uint8)
        v = np.empty_like(u)
        rc = self.lib.hl_amd_get_recon(self._h, y.ctypes.data, u.ctypes.data, v.ctypes.data)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_get_recon")
        return y, u, v

    def set_timing(self, on: bool):
        self.lib.hl_amd_set_timing(self._h, 1 if on else 0)

    def timing_ms(self):
        a = (ctypes.c_float * 4)()
        self.lib.hl_amd_get_timing(self._h, a)
        return list(a)

    def last_reruns(self) -> int:
        return self.lib.hl_amd_last_reruns(self._h)

    def last_chain_walks(self) -> int:
        """resolve_chain walks of the last pipelined run (diagnostics)"""
        return self.lib.hl_amd_last_chain_walks(self._h)

    def profile_counters(self, n: int = 32):
        a = (ctypes.c_ulonglong * n)()
        self.lib.hl_amd_profile_counters(self._h, a, n)
        return list(a)

    def debug_records(self, k: int):
        """MbRecord structs of picture k of the last encode call (numpy
        structured array, one element per macroblock), or None when the
        call did not keep them."""
        import numpy as np

        if not hasattr(self.lib, "hl_amd_debug_records"):
            return None
        nmb = (self.width // 16) * (self.height // 16)
        dt = MB_RECORD
        if self.lib.hl_amd_record_size() == MB_RECORD.itemsize + 32:  # diagnostic build (HL_DIAG_INPUTS)
            dt = np.dtype(MB_RECORD.descr + [("dbg", "<u4", 8)])
        assert self.lib.hl_amd_record_size() == dt.itemsize
        out = np.zeros(nmb, dt)
        rc = self.lib.hl_amd_debug_records(self._h, k, out.ctypes.data, out.nbytes)
        if rc == HL_AMD_ERROR_INVALID_STATE:
            return None
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_debug_records")
        return out

    def debug_chain(self, k: int):
        """MbChain records (s_in, s_out, dep, fresh, spec per macroblock) of
        picture k of the last encode call, as an (nmb, 5) int32 array."""
        import numpy as np

        if not hasattr(self.lib, "hl_amd_debug_chain"):
            return None
        nmb = (self.width // 16) * (self.height // 16)
        out = np.zeros((nmb, 5), np.int32)
        rc = self.lib.hl_amd_debug_chain(self._h, k, out.ctypes.data, out.nbytes)
        if rc == HL_AMD_ERROR_INVALID_STATE:
            return None
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_debug_chain")
        return out

    def debug_recon(self, k: int):
        """Reconstructed planes of picture k of the last encode call,
        concatenated Y|U|V (None when not kept)."""
        import numpy as np

        if not hasattr(self.lib, "hl_amd_debug_recon"):
            return None
        n = self.width * self.height
        out = np.zeros(n * 3 // 2, np.uint8)
        rc = self.lib.hl_amd_debug_recon(self._h, k, out.ctypes.data, out.ctypes.data + n, out.ctypes.data + n + n // 4)
        if rc == HL_AMD_ERROR_INVALID_STATE:
            return None
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_debug_recon")
        return out

    def last_mb_launches(self) -> int:
        return self.lib.hl_amd_last_mb_launches(self._h)

    def last_batch_stats(self) -> dict:
        """How the last encode call ran (hl_amd_last_batch_stats): pipelined
        runs, pictures on the per-picture path, runs that fell back to it,
        bounded waits that gave up, in-kernel rdo.Single_ctr walks."""
        a = (ctypes.c_int32 * 5)()
        rc = self.lib.hl_amd_last_batch_stats(self._h, a)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_last_batch_stats")
        return dict(zip(("runs", "per_picture", "fallbacks", "waits_gave_up", "chain_walks"), list(a)))

    def set_intra_helpers(self, enable: bool) -> None:
        rc = self.lib.hl_amd_set_intra_helpers(self._h, 1 if enable else 0)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_set_intra_helpers")

    def last_helper_stats(self) -> dict:
        """How the last encode call's intra fallbacks ran
        (hl_amd_last_helper_stats): helper Intra4x4 decisions kept, rejected,
        helpers no workgroup had claimed in time."""
        a = (ctypes.c_int32 * 3)()
        rc = self.lib.hl_amd_last_helper_stats(self._h, a)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_last_helper_stats")
        r = dict(zip(("i4_kept", "i4_rejected", "taken_over"), list(a)))
        if hasattr(self.lib, "hl_amd_last_fam3_stats"):
            b = (ctypes.c_int32 * 2)()
            if self.lib.hl_amd_last_fam3_stats(self._h, b) == HL_AMD_SUCCESS:
                r["fam3_kept"], r["fam3_rejected"] = b[0], b[1]
        return r


class SvcEncoder(Encoder):
    """Spatial SVC stream (hl_codec_add_layer + one encode per layer and
    access unit, base first): layer l is (width << l) x (height << l)."""

    def __init__(self, width: int, height: int, layers: int, qp: int = 28, me_range: int = 16, deblock: int = 1, gop_size: int = 30,
                 me_early_term: int = 0, device: int = 0, first: int = 0, last: int = -1):
        super().__init__(width, height, qp, me_range, deblock, gop_size, me_early_term, device)
        self.layers = layers
        for l in range(layers):
            rc = self.lib.hl_amd_add_layer(self._h, width << l, height << l)
            if rc != HL_AMD_SUCCESS:
                raise HlAmdError(rc, "hl_amd_add_layer")
        self.first, self.last = first, (layers - 1 if last < 0 else last)
        if (self.first, self.last) != (0, layers - 1):
            rc = self.lib.hl_amd_set_layer_range(self._h, self.first, self.last)
            if rc != HL_AMD_SUCCESS:
                raise HlAmdError(rc, "hl_amd_set_layer_range")

    def size(self, layer: int):
        return self.width << layer, self.height << layer

    def encode_layer(self, layer: int, y, u, v) -> EncodeResult:
        """One layer's frame from host memory (numpy uint8 planes)."""
        import numpy as np

        w, h = self.size(layer)
        ys = [np.ascontiguousarray(p, dtype=np.uint8) for p in (y, u, v)]
        if ys[0].size != w * h or ys[1].size != w * h // 4 or ys[2].size != ys[1].size:
            raise HlAmdError(HL_AMD_ERROR_INVALID_FORMAT, "encode_layer (plane sizes)")
        r = _Result()
        rc = self.lib.hl_amd_encode_layer(self._h, w, h, ys[0].ctypes.data, ys[1].ctypes.data, ys[2].ctypes.data, 0, ctypes.byref(r))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_layer")
        return self._result(r)

    def encode_layer_device(self, layer: int, y_ptr: int, u_ptr: int, v_ptr: int, collect: bool = True):
        w, h = self.size(layer)
        r = _Result()
        rc = self.lib.hl_amd_encode_layer(self._h, w, h, ctypes.c_void_p(y_ptr), ctypes.c_void_p(u_ptr), ctypes.c_void_p(v_ptr), 1,
                                          ctypes.byref(r))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_layer")
        return self._result(r) if collect else r.data_size

    def layer_recon(self, layer: int):
        import numpy as np

        w, h = self.size(layer)
        out = np.empty(w * h * 3 // 2, np.uint8)
        n = w * h
        rc = self.lib.hl_amd_get_layer_recon(self._h, layer, out.ctypes.data, out.ctypes.data + n, out.ctypes.data + n + n // 4)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_get_layer_recon")
        return out

    def unpinned(self) -> int:
        return self.lib.hl_amd_svc_unpinned(self._h)

    def layer_state_bytes(self, layer: int) -> int:
        return self.lib.hl_amd_layer_state_bytes(self._h, layer)

    def export_layer(self, layer: int, dst_ptr: int):
        rc = self.lib.hl_amd_export_layer(self._h, layer, ctypes.c_void_p(dst_ptr))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_export_layer")

    def import_layer(self, layer: int, src_ptr: int):
        rc = self.lib.hl_amd_import_layer(self._h, layer, ctypes.c_void_p(src_ptr))
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_import_layer")

    def layer_ms(self) -> float:
        return self.lib.hl_amd_svc_layer_ms(self._h)

    def encode_layers_batch_device(self, ptrs):
        """n access units of every layer resident in HBM: ptrs[l][i] =
        (y_ptr, u_ptr, v_ptr) of layer l's frame of access unit i.  Returns
        one EncodeResult per access unit (hl_amd_encode_layers_batch)."""
        L, n = len(ptrs), len(ptrs[0])
        flat = (ctypes.c_void_p * (3 * L * n))(*[ptrs[l][i][c] for l in range(L) for i in range(n) for c in range(3)])
        res = (_Result * n)()
        rc = self.lib.hl_amd_encode_layers_batch(self._h, n, L, flat, res)
        if rc != HL_AMD_SUCCESS:
            raise HlAmdError(rc, "hl_amd_encode_layers_batch")
        return [self._result(r) for r in res]
