"""Host-side mirror of hartallo's codec API for the H.264 encode path.

Same names, argument meaning and error behaviour as the reference's C API
(include/hartallo/hl_codec.h:173-195, source/hl_codec.c:24-229,
include/hartallo/hl_frame.h:278-291), so code and tests written against
hl_codec_encode read the same here:

    plugin = hl_codec_plugin_find(HL_CODEC_TYPE_H264)
    codec = hl_codec_create(plugin)
    codec.qp, codec.gop_size, codec.me_range, codec.deblock_flag = 28, 30, 16, 1
    frame = hl_frame_video_create(); hl_frame_video_fill(frame, W, H, buf)
    result = hl_codec_result_create()
    err = hl_codec_encode(codec, frame, result)     # HL_ERROR_SUCCESS == 0
    if result.type & HL_CODEC_RESULT_TYPE_HDR: out += codec.hdr_bytes
    out += b"\\0\\0\\1" + result.data_ptr

The encoder behind it is the gfx950 library (libhartallo_amd.so).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from ._lib import Encoder, HlAmdError

# HL_ERROR_T (hl_types.h:101-122)
HL_ERROR_SUCCESS = 0
HL_ERROR_INVALID_PARAMETER = 1
HL_ERROR_INVALID_STATE = 3
HL_ERROR_INVALID_FORMAT = 4
HL_ERROR_NOT_IMPLEMENTED = 7
HL_ERROR_NOT_FOUND = 6
# HL_CODEC_TYPE_T / HL_CODEC_RESULT_TYPE_T (hl_types.h:124-163)
HL_CODEC_TYPE_H264 = 1
HL_CODEC_RESULT_TYPE_NONE = 0
HL_CODEC_RESULT_TYPE_DATA = 1
HL_CODEC_RESULT_TYPE_HDR = 2
HL_VIDEO_CHROMA_YUV420 = 0


@dataclass
class hl_codec_plugin_def_t:  # noqa: N801  (reference type name)
    type: int = HL_CODEC_TYPE_H264
    description: str = "H.264 AVC encoder (gfx950 HIP)"


_PLUGINS = [hl_codec_plugin_def_t()]


def hl_codec_plugin_find(codec_type: int):
    """hl_codec_plugin_find (hl_codec.c:215-229): first plugin of the type."""
    for p in _PLUGINS:
        if p.type == codec_type:
            return p
    return None


@dataclass
class hl_codec_t:  # noqa: N801
    """The hl_codec_t fields the encoder reads (hl_codec.h:33-80)."""

    plugin: hl_codec_plugin_def_t
    width: int = 0
    height: int = 0
    qp: int = 24
    gop_size: int = 25
    me_range: int = 16
    deblock_flag: int = 1
    me_early_term_flag: int = 1  # reference default (hl_types.h:67)
    fps_num: int = 1             # fps (hl_codec.c:37-38): 1/15
    fps_den: int = 15
    rc_bitrate: int = -1         # rate control when > 0 (hl_types.h:59-64 defaults)
    rc_basicunit: int = -1
    rc_qp_min: int = -1
    rc_qp_max: int = -1
    threads_count: int = 1
    max_ref_frame: int = 1
    device: int = 0
    hdr_bytes: bytes = b""
    _enc: Encoder = field(default=None, repr=False)


@dataclass
class hl_frame_video_t:  # noqa: N801
    width: int = 0
    height: int = 0
    chroma: int = HL_VIDEO_CHROMA_YUV420
    data_ptr: tuple = ()


@dataclass
class hl_codec_result_t:  # noqa: N801
    type: int = HL_CODEC_RESULT_TYPE_NONE
    data_ptr: bytes = b""
    data_size: int = 0
    width: int = 0
    height: int = 0


def hl_codec_create(plugin) -> hl_codec_t:
    if plugin is None:
        raise HlAmdError(HL_ERROR_INVALID_PARAMETER, "hl_codec_create")
    return hl_codec_t(plugin=plugin)


def hl_codec_result_create() -> hl_codec_result_t:
    return hl_codec_result_t()


def hl_frame_video_create() -> hl_frame_video_t:
    return hl_frame_video_t()


def hl_frame_video_fill(frame: hl_frame_video_t, width: int, height: int, buf) -> int:
    """hl_frame_video_fill for planar YUV420 (hl_frame.c): buf holds Y|U|V."""
    a = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf.reshape(-1)
    n = width * height
    if a.size < n * 3 // 2:
        return HL_ERROR_INVALID_PARAMETER
    frame.width, frame.height = width, height
    frame.data_ptr = (a[:n], a[n:n + n // 4], a[n + n // 4:n * 3 // 2])
    return HL_ERROR_SUCCESS


def hl_codec_encode(codec: hl_codec_t, frame: hl_frame_video_t, result: hl_codec_result_t) -> int:
    """hl_codec_encode (hl_codec.c:152-159) routed to the gfx950 plugin."""
    if codec is None or frame is None or result is None:
        return HL_ERROR_INVALID_PARAMETER
    if frame.width % 16 or frame.height % 16:
        return HL_ERROR_INVALID_FORMAT  # hl_codec_264.c:437-438
    if codec._enc is None or (codec.width, codec.height) != (frame.width, frame.height):
        if codec.threads_count > 1:  # threads_count slices per picture (hl_codec_264.c:571): one slice here; <= 0 is 1 (hl_codec_264.c:1053-1054)
            return HL_ERROR_NOT_IMPLEMENTED
        try:
            codec._enc = Encoder(frame.width, frame.height, codec.qp, codec.me_range, codec.deblock_flag, codec.gop_size,
                                 codec.me_early_term_flag, codec.device)
            codec._enc.set_max_ref_frame(codec.max_ref_frame)  # SPS/PPS fields (hl_codec_264_sps.c:620-636)
            if codec.rc_bitrate > 0:  # hl_codec_264.c:719-742
                codec._enc.set_rate_control(codec.rc_bitrate, codec.fps_num, codec.fps_den, codec.rc_basicunit, codec.rc_qp_min,
                                            codec.rc_qp_max)
        except HlAmdError as e:
            return e.code
        codec.width, codec.height = frame.width, frame.height
    try:
        r = codec._enc.encode(*frame.data_ptr)
    except HlAmdError as e:
        return e.code
    result.type = r.type
    result.data_ptr = r.data
    result.data_size = len(r.data)
    result.width, result.height = frame.width, frame.height
    if r.type & HL_CODEC_RESULT_TYPE_HDR:
        codec.hdr_bytes = r.hdr
    return HL_ERROR_SUCCESS
