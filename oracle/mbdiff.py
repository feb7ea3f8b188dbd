"""mbdiff.py -- TEST INFRASTRUCTURE: compare two encoder dumps (ref_enc vs
hlenc_oracle vs the HIP encoder) frame by frame and MB by MB.

usage: python oracle/mbdiff.py W H prefixA prefixB [max_reports]
"""
import sys

import numpy as np

FIELDS = [
    ("FLAGS", 0, 1), ("MB_TYPE", 1, 1), ("SUB_MB_TYPE", 2, 4), ("NUM_MB_PART", 6, 1), ("MVL0", 7, 32), ("MVD", 39, 32),
    ("CBP_L4x4", 71, 1), ("CBP", 72, 1), ("CBP_L", 73, 1), ("CBP_C", 74, 1), ("CBP_CAC", 75, 2), ("CBP_CDC", 77, 2),
    ("I16_MODE", 79, 1), ("I4_MODE", 80, 16), ("CHROMA_MODE", 96, 1), ("PREV_FLAG", 97, 16), ("REM_MODE", 113, 16),
    ("QPY", 129, 1), ("TC_LUMA", 130, 16), ("TC_CAC", 146, 8), ("LUMA_LEVEL", 154, 256), ("I16_DC", 410, 16),
    ("I16_AC", 426, 256), ("CHROMA_DC", 682, 8), ("CHROMA_AC", 690, 128), ("ETYPE", 818, 1), ("MVL0_CAP", 819, 32),
]
STRIDE = 864


def main():
    W, H = int(sys.argv[1]), int(sys.argv[2])
    a, b = sys.argv[3], sys.argv[4]
    maxrep = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    nmb = (W // 16) * (H // 16)
    fs = W * H * 3 // 2
    ra = np.fromfile(a + ".mbs", dtype=np.int32).reshape(-1, nmb, STRIDE)
    rb = np.fromfile(b + ".mbs", dtype=np.int32).reshape(-1, nmb, STRIDE)
    ya = np.fromfile(a + ".rec.yuv", dtype=np.uint8).reshape(-1, fs)
    yb = np.fromfile(b + ".rec.yuv", dtype=np.uint8).reshape(-1, fs)
    sa = open(a + ".264", "rb").read()
    sb = open(b + ".264", "rb").read()
    print(f"stream: {len(sa)} vs {len(sb)} bytes, equal={sa == sb}")
    if sa != sb:
        i = next((k for k in range(min(len(sa), len(sb))) if sa[k] != sb[k]), min(len(sa), len(sb)))
        print(f"  first stream diff at byte {i}")
    nf = min(len(ra), len(rb))
    rep = 0
    for f in range(nf):
        recdiff = np.nonzero(ya[f] != yb[f])[0]
        if len(recdiff):
            p = recdiff[0]
            if p < W * H:
                print(f"frame {f}: recon differs, first luma ({p % W},{p // W}) MB {(p // W // 16) * (W // 16) + (p % W) // 16}")
            else:
                print(f"frame {f}: recon differs first at chroma offset {p - W * H}")
        for m in range(nmb):
            diffs = []
            for name, off, n in FIELDS:
                if not np.array_equal(ra[f, m, off:off + n], rb[f, m, off:off + n]):
                    diffs.append(f"{name}: {ra[f, m, off:off + n].tolist()} vs {rb[f, m, off:off + n].tolist()}")
            if diffs:
                print(f"frame {f} MB {m} ({m % (W // 16)},{m // (W // 16)}):")
                for d in diffs:
                    print("   ", d[:400])
                rep += 1
                if rep >= maxrep:
                    return
        if rep:
            return
    print("all MB records equal" if rep == 0 else "")


if __name__ == "__main__":
    main()
