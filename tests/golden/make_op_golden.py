"""Op-level goldens from the reference's own per-block kernels.

oracle/_ref/ref_ops (oracle/ref_ops.c, linked with the reference library
oracle/Makefile builds from /root/reference's sources) runs the reference's
transform / quantiser / dequantiser / IDCT, CAVLC residual writer, luma
interpolation and baseline deblocking filter steps on seeded vectors made
here; inputs and the reference's outputs are stored as
tests/golden/ops_<op>.npz (numpy, no pickles).  tests/test_gpu_ops.py runs
the gfx950 kernels (the quad / 16-lane pipelines, cavlc_block, k_planes +
pred_luma4x4, deblock_line; tests/gpu_unit/libhl_unit.so) on the same inputs.

Run in the build container (needs oracle/_ref/ref_ops):
    python tests/golden/make_op_golden.py
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_OPS = os.path.join(ROOT, "oracle", "_ref", "ref_ops")


def run(op, inp, out_dtype):
    with tempfile.TemporaryDirectory() as td:
        a, b = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(a, "wb") as f:
            f.write(inp)
        subprocess.run([REF_OPS, op, a, b], check=True)
        return np.fromfile(b, dtype=out_dtype)


def blocks(rng, n):
    """src / pred 4x4 blocks: sparse, small, medium and full-range residuals
    (the distribution of tests/test_gpu_unit.py)."""
    pred = rng.integers(0, 256, (n, 16))
    kind = rng.integers(0, 4, n)
    amp = np.choose(kind, [2, 6, 30, 255])
    res = (rng.integers(-255, 256, (n, 16)) * amp[:, None]) // 255
    res[kind == 0] *= rng.integers(0, 2, (int((kind == 0).sum()), 16))
    src = np.clip(pred + res, 0, 255)
    return src.astype(np.uint8), pred.astype(np.uint8)


def make_xform(rng):
    """Every QP 0..51, inter and intra rounding, 96 blocks each."""
    xin = np.dtype([("src", "u1", 16), ("pred", "u1", 16), ("qp", "<i4"), ("intra", "<i4")])
    xout = np.dtype([("q", "<i4", 16), ("rec", "u1", 16)])
    recs = []
    for qp in range(52):
        for intra in (0, 1):
            s, p = blocks(rng, 96)
            r = np.zeros(96, xin)
            r["src"], r["pred"], r["qp"], r["intra"] = s, p, qp, intra
            recs.append(r)
    recs = np.concatenate(recs)
    out = run("xform", recs.tobytes(), xout)
    return dict(src=recs["src"], pred=recs["pred"], qp=recs["qp"], intra=recs["intra"], q=out["q"], rec=out["rec"])


def level_lists(rng, n, maxn):
    """Scan-order level lists: every TotalCoeff, trailing ones, magnitudes
    from 1 to escape-code range (|level| <= 2000: an 8-bit residual at QP 0)."""
    lv = np.zeros((n, 16), np.int32)
    for i in range(n):
        tc = int(rng.integers(0, maxn + 1))
        pos = np.sort(rng.choice(maxn, tc, replace=False))
        style = int(rng.integers(0, 5))
        if style == 0:
            mag = np.ones(tc, np.int32)
        elif style == 1:
            mag = rng.integers(1, 4, tc)
        elif style == 2:
            mag = rng.integers(1, 20, tc)
        elif style == 3:
            mag = np.where(rng.random(tc) < 0.3, rng.integers(1, 2001, tc), rng.integers(1, 3, tc))
        else:  # large first levels (suffixLength escalation), trailing ones at the end
            mag = np.sort(rng.integers(1, 300, tc))[::-1].copy()
            mag[-min(tc, 3):] = 1
        sign = np.where(rng.random(tc) < 0.5, -1, 1)
        lv[i, pos] = mag * sign
    return lv


def make_cavlc(rng):
    """Luma 4x4 (16), Intra16x16 AC (15), chroma AC (15) at nC 0..16, the AC
    list with the RDO's (0, 15, 16) bounds, and chroma DC (4, nC -1)."""
    cin = np.dtype([("kind", "<i4"), ("nC", "<i4"), ("level", "<i4", 16)])
    cout = np.dtype([("nbits", "<i4"), ("bits", "u1", 96)])
    recs = []
    for kind, maxn in ((0, 16), (1, 15), (3, 15), (4, 15)):  # (4: the AC list as the RDO prices it, rdo.c:1676)
        for nc in (0, 1, 2, 3, 4, 5, 7, 8, 9, 12, 16):
            r = np.zeros(96, cin)
            r["kind"], r["nC"], r["level"] = kind, nc, level_lists(rng, 96, maxn)
            recs.append(r)
    r = np.zeros(512, cin)
    r["kind"], r["nC"], r["level"] = 2, -1, level_lists(rng, 512, 4)
    recs.append(r)
    recs = np.concatenate(recs)
    out = run("cavlc", recs.tobytes(), cout)
    return dict(kind=recs["kind"], nC=recs["nC"], level=recs["level"], nbits=out["nbits"], bits=out["bits"])


def make_lpred(rng):
    """16x16 luma predictions at every quarter-pel phase, every macroblock of
    a 96x64 picture (interior and edges), motion reaching 24 samples beyond
    the picture."""
    W, H = 96, 64
    yy, xx = np.mgrid[0:H, 0:W]
    luma = np.clip(128 + 60 * np.sin(xx / 7.0) * np.cos(yy / 5.0) + rng.integers(-40, 41, (H, W)), 0, 255).astype(np.uint8)
    pin = np.dtype([("mbx", "<i4"), ("mby", "<i4"), ("mvx", "<i4"), ("mvy", "<i4")])
    recs = []
    for ph in range(16):
        for mby in range(H // 16):
            for mbx in range(W // 16):
                r = np.zeros(3, pin)
                r["mbx"], r["mby"] = mbx, mby
                r["mvx"] = rng.integers(-24, 25, 3) * 4 + (ph & 3)
                r["mvy"] = rng.integers(-24, 25, 3) * 4 + (ph >> 2)
                recs.append(r)
    recs = np.concatenate(recs)
    hdr = np.array([W, H], "<i4").tobytes() + luma.tobytes()
    out = run("lpred", hdr + recs.tobytes(), np.uint8).reshape(-1, 16, 16)
    return dict(W=np.int32(W), H=np.int32(H), luma=luma, mbx=recs["mbx"], mby=recs["mby"], mvx=recs["mvx"], mvy=recs["mvy"], pred=out)


def make_dblk(rng):
    """Eight lines across one edge for every bS 1..4 x indexA 0..51, luma and
    chroma: smooth sides with a step, amplitudes around the alpha / beta
    thresholds so that lines are filtered and bypassed."""
    din = np.dtype([("p", "u1", (4, 8)), ("q", "u1", (4, 8)), ("bS", "<i4"), ("indexA", "<i4"), ("chroma", "<i4")])
    dout = np.dtype([("p", "u1", (3, 8)), ("q", "u1", (3, 8))])
    recs = []
    for chroma in (0, 1):
        for bs in (1, 2, 3, 4):
            for ia in range(52):
                r = np.zeros(6, din)
                r["bS"], r["indexA"], r["chroma"] = bs, ia, chroma
                base = rng.integers(0, 256, (6, 1, 8))
                step = rng.integers(-40, 41, (6, 1, 8)) * rng.integers(0, 2, (6, 1, 1))
                noise = rng.integers(0, 3, (6, 1, 1)) * 4 + 1
                p = base + rng.integers(-1, 2, (6, 4, 8)) * rng.integers(0, noise + 1, (6, 4, 8))
                q = base + step + rng.integers(-1, 2, (6, 4, 8)) * rng.integers(0, noise + 1, (6, 4, 8))
                r["p"], r["q"] = np.clip(p, 0, 255), np.clip(q, 0, 255)
                recs.append(r)
    recs = np.concatenate(recs)
    out = run("dblk", recs.tobytes(), dout)
    return dict(p_in=recs["p"], q_in=recs["q"], bS=recs["bS"], indexA=recs["indexA"], chroma=recs["chroma"], p_out=out["p"], q_out=out["q"])


def main():
    if not os.path.exists(REF_OPS):
        sys.exit(f"{REF_OPS} missing: run `make -C oracle ref` where /root/reference exists")
    for name, fn, seed in (("xform", make_xform, 601), ("cavlc", make_cavlc, 602), ("lpred", make_lpred, 603), ("dblk", make_dblk, 604)):
        d = fn(np.random.default_rng(seed))
        np.savez_compressed(os.path.join(HERE, f"ops_{name}.npz"), **d)
        print(name, {k: getattr(v, "shape", ()) for k, v in d.items()})


if __name__ == "__main__":
    main()
