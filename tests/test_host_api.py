"""Host-side mirror of the reference codec API (hartallo_amd/hl_codec.py) and
the synthetic input generator -- CPU only."""
import numpy as np
import pytest

from hartallo_amd import hl_codec as hc
from hartallo_amd import synth


def test_plugin_find_and_create():
    p = hc.hl_codec_plugin_find(hc.HL_CODEC_TYPE_H264)
    assert p is not None and p.type == hc.HL_CODEC_TYPE_H264
    assert hc.hl_codec_plugin_find(99) is None
    c = hc.hl_codec_create(p)
    assert (c.threads_count, c.max_ref_frame) == (1, 1)
    with pytest.raises(Exception):
        hc.hl_codec_create(None)


def test_frame_fill_and_format_errors():
    f = hc.hl_frame_video_create()
    assert hc.hl_frame_video_fill(f, 352, 288, np.zeros(352 * 288, np.uint8)) == hc.HL_ERROR_INVALID_PARAMETER
    assert hc.hl_frame_video_fill(f, 352, 288, np.zeros(352 * 288 * 3 // 2, np.uint8)) == hc.HL_ERROR_SUCCESS
    assert [p.size for p in f.data_ptr] == [352 * 288, 352 * 288 // 4, 352 * 288 // 4]
    c = hc.hl_codec_create(hc.hl_codec_plugin_find(hc.HL_CODEC_TYPE_H264))
    f2 = hc.hl_frame_video_create()
    hc.hl_frame_video_fill(f2, 1920, 1080, np.zeros(1920 * 1080 * 3 // 2, np.uint8))
    assert hc.hl_codec_encode(c, f2, hc.hl_codec_result_create()) == hc.HL_ERROR_INVALID_FORMAT
    c.threads_count = 2  # the reference codes threads_count slices per picture (hl_codec_264.c:571): refused
    assert hc.hl_codec_encode(c, f, hc.hl_codec_result_create()) == hc.HL_ERROR_NOT_IMPLEMENTED
    import torch

    if not torch.cuda.is_available():  # max_ref_frame is forwarded; without a GPU the encoder refuses loudly
        # threads_count <= 0 counts as 1 (hl_codec_264.c:1053-1054), as in the C plugin: not refused as slices
        for tc in (1, 0, -3):
            c.threads_count, c.max_ref_frame = tc, 4
            assert hc.hl_codec_encode(c, f, hc.hl_codec_result_create()) not in (hc.HL_ERROR_SUCCESS, hc.HL_ERROR_NOT_IMPLEMENTED)


def test_synth_is_deterministic():
    a = synth.clip(64, 32, 3, 5)
    b = synth.clip(64, 32, 3, 5)
    c = synth.clip(64, 32, 3, 6)
    assert a.shape == (3, 64 * 32 * 3 // 2) and a.dtype == np.uint8
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    y0 = a[0, :64 * 32].reshape(32, 64)
    u0 = a[0, 64 * 32:64 * 32 + 16 * 32].reshape(16, 32)
    assert np.array_equal(u0, y0[::2, ::2] // 2 + 64)
