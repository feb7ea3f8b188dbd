"""Spatial-SVC goldens of the reference encoder (tests/golden/svc_golden.json).

Each workload is encoded by oracle/_ref/ref_svc -- the reference's own C
sources driven as an SVC encoder through its public API (hl_codec_add_layer
per layer, then one hl_codec_encode per layer and frame, base first, as
source/test_encoder.c:151-202 does with HL_TEST_ENCODER_SVC_ENABLED) -- on
hartallo_amd.synth.svc_clips input (the top layer is synth.clip, each layer
below is its 2x2 box-average downscale).  Kept per workload:
  au_md5[i], au_bytes[i]   MD5 / size of what the harness writes for access
                           unit i: header NAL units when signalled (every
                           layer's first call), then 00 00 01 + the result
                           bytes of the last layer's call
  recon_md5[l][i]          MD5 of layer l's reconstructed (deblocked) picture
                           after access unit i
  intra_in_p               reference-layer intra macroblocks in P pictures
                           (outside the pinned scope, hl_svc.h); 0 for all
Workloads that are small also keep the whole stream (<name>.264).

Run in the build container (needs oracle/_ref/ref_svc):
  python tests/golden/make_svc_golden.py [name ...]
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from hartallo_amd import synth  # noqa: E402

REF_SVC = os.path.join(ROOT, "oracle", "_ref", "ref_svc")
OUT = os.path.join(HERE, "svc_golden.json")
MBR_STRIDE = 864  # oracle/mbrec.h

# name: (W0, H0, layers, frames, qp, me_range, deblock, gop, early_term, seed, keep_stream)
WORKLOADS = {
    "svc3_64x48_qp30_gop3": (64, 48, 3, 5, 30, 8, 1, 3, 0, 5, True),
    "svc2_qcif_qp36_nodb_gop2": (176, 144, 2, 4, 36, 16, 0, 2, 0, 6, True),
    "svc2_qcif_qp28_db": (176, 144, 2, 4, 28, 16, 1, 30, 0, 3, False),
    "svc2_et_qcif_qp24": (176, 144, 2, 3, 24, 16, 1, 30, 1, 9, False),
    # BASELINE config 4 as the reference expresses it:
    # dyadic 480x272 / 960x544 / 1920x1088, IPPP GOP 30, QP28, ME 16, deblocking,
    # 31 frames (across the second IDR)
    "c4_svc3_480x272_s41": (480, 272, 3, 31, 28, 16, 1, 30, 0, 41, False),
}


def md5(b) -> str:
    return hashlib.md5(b).hexdigest()


def encode(name):
    w0, h0, L, n, qp, mer, db, gop, et, seed, keep = WORKLOADS[name]
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, n, seed)
    with tempfile.TemporaryDirectory() as td:
        ins = []
        for l in range(L):
            p = os.path.join(td, f"in{l}.yuv")
            clips[l].tofile(p)
            ins.append(p)
        pre = os.path.join(td, "o")
        r = subprocess.run([REF_SVC, str(L), str(w0), str(h0), str(n), str(qp), str(mer), str(db), str(gop), str(et), pre] + ins,
                           check=True, capture_output=True, text=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
        stream = open(pre + ".264", "rb").read()
        ends = [int(v) for v in open(pre + ".idx").read().split()]
        starts = [0] + ends[:-1]
        recon = []
        for l in range(L):
            fs = (w0 << l) * (h0 << l) * 3 // 2
            rec = np.fromfile(f"{pre}.L{l}.rec.yuv", np.uint8).reshape(-1, fs)
            recon.append([md5(rec[i].tobytes()) for i in range(rec.shape[0])])
        # intra MBs of reference layers (all but the top) in P pictures
        intra_in_p = 0
        for l in range(L - 1):
            nmb = ((w0 << l) // 16) * ((h0 << l) // 16)
            recs = np.fromfile(f"{pre}.L{l}.mbs", np.int32).reshape(-1, nmb, MBR_STRIDE)
            for i in range(recs.shape[0]):
                if i % gop:
                    intra_in_p += int((recs[i, :, 0] & 1).sum())
        if keep:
            open(os.path.join(HERE, name + ".264"), "wb").write(stream)
    return name, {
        "w0": w0, "h0": h0, "layers": L, "frames": info["frames"], "qp": qp, "me_range": mer, "deblock": db, "gop": gop,
        "early_term": et, "seed": seed, "stream": (name + ".264") if keep else None,
        "au_md5": [md5(stream[s:e]) for s, e in zip(starts, ends)],
        "au_bytes": [e - s for s, e in zip(starts, ends)],
        "recon_md5": recon, "intra_in_p": intra_in_p, "stream_md5": md5(stream),
        "ref_seconds": info["seconds"],
    }


def main():
    names = sys.argv[1:] or list(WORKLOADS)
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    with ThreadPoolExecutor(max_workers=min(4, len(names))) as ex:
        for name, d in ex.map(encode, names):
            data[name] = d
            print(name, d["frames"], "AUs", sum(d["au_bytes"]), "bytes, intra_in_p", d["intra_in_p"], flush=True)
    data = {k: data[k] for k in WORKLOADS if k in data}
    json.dump(data, open(OUT, "w"), indent=1)


if __name__ == "__main__":
    main()
