"""Synthetic planar YUV420 input, seeded.

A blurred random texture translated by (2t + t mod 3, t) pixels per frame
plus uniform noise in [-3, 3]; U = Y/2 + 64 and V = 255 - Y/2 on the 2x
subsampled luma.  Deterministic for a given (width, height, frames, seed).
"""
from __future__ import annotations

import numpy as np


def _blur5(a: np.ndarray) -> np.ndarray:
    # separable 5-tap box filter with zero padding ('same' convolution)
    p = np.pad(a, ((0, 0), (2, 2)))
    a = (p[:, 0:-4] + p[:, 1:-3] + p[:, 2:-2] + p[:, 3:-1] + p[:, 4:]) / np.float32(5.0)
    p = np.pad(a, ((2, 2), (0, 0)))
    return (p[0:-4] + p[1:-3] + p[2:-2] + p[3:-1] + p[4:]) / np.float32(5.0)


def frames(width: int, height: int, n: int, seed: int):
    """Yields n frames as (y, u, v) uint8 planes."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (height + 8 * n + 16, width + 8 * n + 16)).astype(np.float32)
    base = _blur5(base)
    for t in range(n):
        dx = 2 * t + (t % 3)
        dy = t
        y = np.clip(base[dy:dy + height, dx:dx + width] + rng.integers(-3, 4, (height, width)), 0, 255).astype(np.uint8)
        s = y[::2, ::2]
        u = (s // 2 + 64).astype(np.uint8)
        v = (255 - s // 2).astype(np.uint8)
        yield y, u, v


def clip(width: int, height: int, n: int, seed: int) -> np.ndarray:
    """n frames concatenated as planar Y|U|V bytes, shape (n, w*h*3/2)."""
    return np.stack([np.concatenate([y.ravel(), u.ravel(), v.ravel()]) for y, u, v in frames(width, height, n, seed)])


def _down2(p: np.ndarray) -> np.ndarray:
    # 2x2 box average with rounding
    a = p.astype(np.uint16)
    return ((a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2] + 2) >> 2).astype(np.uint8)


def svc_clips(width: int, height: int, layers: int, n: int, seed: int) -> list:
    """Spatial-SVC input: the top layer is clip(width, height, n, seed); layer
    l below it is the 2x2 box-average downscale of layer l+1 (planes
    separately).  Returns [clip of layer 0 (smallest), ..., clip of the top
    layer], each shaped (n, w_l*h_l*3/2)."""
    top = clip(width, height, n, seed)
    out = [top]
    w, h = width, height
    for _ in range(layers - 1):
        fs = w * h
        cur = out[0]
        nxt = []
        for f in range(n):
            y = cur[f, :fs].reshape(h, w)
            u = cur[f, fs:fs + fs // 4].reshape(h // 2, w // 2)
            v = cur[f, fs + fs // 4:].reshape(h // 2, w // 2)
            nxt.append(np.concatenate([_down2(y).ravel(), _down2(u).ravel(), _down2(v).ravel()]))
        w, h = w // 2, h // 2
        out.insert(0, np.stack(nxt))
    return out
