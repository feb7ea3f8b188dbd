"""Development tool (CPU, emulator): per picture, how many of the 8x8-family
partitioning helpers' results the macroblocks kept and rejected (f3_verify),
on golden configurations -- the rejection rate of the helpers' entry-value
guess picture by picture.

  python tools/fam3_guess_stats.py [name ...]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

from hl_testlib import GOLDEN_CONFIGS, EmuEncoder, golden_input  # noqa: E402


def main():
    names = sys.argv[1:] or ["cif_ippp_qp31_me8", "qcif_ippp_qp28_db", "w480_h272_qp28_me16"]
    tot = [0, 0]
    cfgs = list(GOLDEN_CONFIGS)
    if "bench" in names:  # the first pictures of the bench stream (1920x1088, seed 11)
        cfgs.append(("bench", 1920, 1088, int(os.environ.get("FRAMES", "4")), 28, 16, 1, 30, 11))
    for cfg in cfgs:
        if cfg[0] not in names:
            continue
        name, w, h, n, qp, mer, db, gop, seed = cfg
        if name == "bench":
            from hartallo_amd import synth

            sys.path.insert(0, ROOT)
            clip = synth.clip(w, h, 150, seed)[:n]
        else:
            clip = golden_input(cfg)
        enc = EmuEncoder(w, h, qp, mer, db, gop)
        enc.lib.emu_set_helper(ctypes.c_void_p(enc.h_), 4)
        prev = [0, 0]
        row = []
        for f in range(n):
            enc.encode(clip[f])
            cur = [enc.lib.emu_helper_fam3(ctypes.c_void_p(enc.h_), k) for k in (0, 1)]
            d = [cur[0] - prev[0], cur[1] - prev[1]]
            prev = cur
            row.append(f"{d[0]}/{d[1]}")
            tot[0] += d[0]
            tot[1] += d[1]
        print(f"{name}: kept/rejected per picture {' '.join(row)}", flush=True)
    print(f"total kept {tot[0]} rejected {tot[1]} ({100.0 * tot[1] / max(1, sum(tot)):.1f} %)")


if __name__ == "__main__":
    main()
