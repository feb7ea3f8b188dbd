"""Repeats the GOP-spanning 1920x1088 pipelined run (tests/test_gpu_pipeline.py
test_batch_1088p_spans_gops) in one process and reports every run whose
stream differs from the same frames encoded one call at a time.

  python tools/stress_spans_gops.py [repeats] [frames] [gop]

Development tool for the pipelined-run parity defect.  Set HL_LIB
to run another build of the library, HL_PIPE=workgroups,reach,window to set
the pipeline geometry.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hartallo_amd import _lib  # noqa: E402

if os.environ.get("HL_LIB"):
    _lib.load_library(os.path.abspath(os.environ["HL_LIB"]))
from hartallo_amd import Encoder, synth  # noqa: E402
from hl_testlib import first_diff, first_record_diff  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    gop = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    w, h = 1920, 1088
    clip = synth.clip(w, h, n, 13)
    dev = torch.from_numpy(np.ascontiguousarray(clip)).cuda()
    torch.cuda.synchronize()
    ny = w * h
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(n)]
    enc = Encoder(w, h, 28, 16, 1, gop)
    ref, ref_recs, ref_chain, ref_pics = [], [], [], []
    for p in ptrs:
        ref.append(enc.encode_device(*p).annexb())
        ref_recs.append(enc.debug_records(0))
        ref_chain.append(enc.debug_chain(0))
        ref_pics.append(enc.debug_recon(0))
    ref_rec = np.concatenate(enc.recon())
    enc.close()
    mbw, mbh = w // 16, h // 16
    wave = sorted(range(mbw * mbh), key=lambda m: ((m % mbw) + 2 * (m // mbw), m // mbw))

    def first_mb(diff_mask):  # first MB in wavefront order with a difference
        for m in wave:
            if diff_mask[m]:
                return f"({m % mbw},{m // mbw})"
        return None

    def pic_diff(a, b):
        n = w * h
        ya, yb = a[:n].reshape(h, w), b[:n].reshape(h, w)
        mb = (ya != yb).reshape(mbh, 16, mbw, 16).any(axis=(1, 3)).ravel()
        ca = a[n:].reshape(2, h // 2, w // 2) != b[n:].reshape(2, h // 2, w // 2)
        mbc = ca.reshape(2, mbh, 8, mbw, 8).any(axis=(0, 2, 4)).ravel()
        return first_mb(mb), first_mb(mbc)
    geometry = tuple(int(v) for v in os.environ["HL_PIPE"].split(",")) if os.environ.get("HL_PIPE") else None
    bad = 0
    for r in range(reps):
        enc = Encoder(w, h, 28, 16, 1, gop)
        if geometry:
            enc.set_pipeline(*geometry)
        if os.environ.get("HL_STRESS_SINGLE"):  # the per-picture path instead of pipelined runs
            out, recs, chains, pics = [], [], [], []
            for p in ptrs:
                out.append(enc.encode_device(*p).annexb())
                recs.append(enc.debug_records(0))
                chains.append(enc.debug_chain(0))
                pics.append(enc.debug_recon(0))
        else:
            out = [x.annexb() for x in enc.encode_batch_device(ptrs)]
            recs = [enc.debug_records(k) for k in range(n)]
        chains = [enc.debug_chain(k) for k in range(n)]
        pics = [enc.debug_recon(k) for k in range(n)]
        reruns = enc.last_reruns()
        recon_ok = np.array_equal(np.concatenate(enc.recon()), ref_rec)
        enc.close()
        diffs = [(f, first_diff(ref[f], out[f]), len(ref[f])) for f in range(n) if ref[f] != out[f]]
        bad += bool(diffs) or not recon_ok
        msg = "ok" if not diffs else f"MISMATCH {diffs}; {first_record_diff(ref_recs, recs, w // 16)}"
        print(f"run {r}: {msg} (recon {'equal' if recon_ok else 'DIFFERS'}, reruns {reruns})", flush=True)
        for f in range(n) if (diffs or not recon_ok) and chains[0] is not None else []:
            ch = first_mb((chains[f] != ref_chain[f]).any(axis=1))
            ly, lc = pic_diff(ref_pics[f], pics[f])
            if ch or ly or lc:
                print(f"   picture {f}: first MB (wavefront order) with a different chain record {ch}, luma recon {ly}, chroma recon {lc}",
                      flush=True)
    print(f"{bad} of {reps} runs differ", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
