"""Regenerates tests/golden/ from the reference encoder itself.

Each configuration in tests/hl_testlib.GOLDEN_CONFIGS (and GOLDEN_ET_CONFIGS,
encoded with me_early_term_flag = 1, GOLDEN_RC_CONFIGS with rate control,
GOLDEN_MRF_CONFIGS with hl_codec_t.max_ref_frame > 1) is synthesised with
hartallo_amd.synth (seeded), encoded by oracle/_ref/ref_enc (the reference's
own C sources compiled by oracle/Makefile, driven through hl_codec_encode as
source/test_encoder.c does), and stored as:
  <name>.264        the reference's Annex-B output
  golden.json       per-config parameters, stream MD5 and per-frame MD5 of
                    the reference's reconstructed (deblocked) pictures

Run in the build container (needs /root/reference):  python tests/golden/make_golden.py [name ...]
With names, only those entries are (re)made and the rest of golden.json --
including make_decoded_golden.py's decoded_md5 fields -- is kept.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402

from hl_testlib import (GOLDEN_CONFIGS, GOLDEN_ET_CONFIGS, GOLDEN_FAIL_CONFIGS, GOLDEN_MRF_CONFIGS, GOLDEN_RC_CONFIGS, REF_ENC,  # noqa: E402
                        golden_input, md5, slice_qps)


def main():
    if not os.path.exists(REF_ENC):
        sys.exit(f"{REF_ENC} missing: run `make -C oracle ref` where /root/reference exists")
    only = set(sys.argv[1:])
    gpath = os.path.join(HERE, "golden.json")
    table = json.load(open(gpath)) if only else {}
    with tempfile.TemporaryDirectory() as td:
        for cfg in GOLDEN_CONFIGS + GOLDEN_ET_CONFIGS + GOLDEN_RC_CONFIGS + GOLDEN_MRF_CONFIGS + GOLDEN_FAIL_CONFIGS:
            name, w, h, n, qp, mer, db, gop, seed = cfg[:9]
            if only and name not in only:
                continue
            et = 1 if cfg in GOLDEN_ET_CONFIGS else 0
            env = dict(os.environ)
            for k in ("HL_REF_RC_BITRATE", "HL_REF_RC_BASICUNIT", "HL_REF_RC_QP_MIN", "HL_REF_RC_QP_MAX", "HL_REF_MAX_REF_FRAME"):
                env.pop(k, None)
            if cfg in GOLDEN_MRF_CONFIGS:  # hl_codec_t.max_ref_frame (ref_harness.c)
                env["HL_REF_MAX_REF_FRAME"] = str(cfg[9])
            if cfg in GOLDEN_RC_CONFIGS:  # rate control: bitrate, basic unit, QP range (ref_harness.c)
                env.update(HL_REF_RC_BITRATE=str(cfg[9]), HL_REF_RC_BASICUNIT=str(cfg[10]), HL_REF_RC_QP_MIN=str(cfg[11]),
                           HL_REF_RC_QP_MAX=str(cfg[12]))
            clip = golden_input(cfg)
            inp = os.path.join(td, name + ".yuv")
            clip.tofile(inp)
            pre = os.path.join(td, name)
            r = subprocess.run([REF_ENC, str(w), str(h), str(n), str(qp), str(mer), str(db), str(gop), str(et), inp, pre, "rec"],
                               stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True, env=env)
            fail = {}
            if cfg in GOLDEN_FAIL_CONFIGS:  # ref_harness.c: "encode err <code> at frame <f>", exit status 4
                m = re.search(r"encode err (\d+) at frame (\d+)", r.stderr)
                assert r.returncode == 4 and m, f"{name}: the reference was expected to fail"
                fail = {"fail_error": int(m.group(1)), "fail_frame": int(m.group(2))}
            elif r.returncode:
                raise subprocess.CalledProcessError(r.returncode, REF_ENC, stderr=r.stderr[-2000:])
            stream = open(pre + ".264", "rb").read()
            rec = np.fromfile(pre + ".rec.yuv", dtype=np.uint8).reshape(-1, w * h * 3 // 2)
            with open(os.path.join(HERE, name + ".264"), "wb") as f:
                f.write(stream)
            table[name] = {
                "width": w, "height": h, "frames": n, "qp": qp, "me_range": mer, "deblock": db, "gop": gop, "seed": seed,
                "early_term": et,
                **({"rc_bitrate": cfg[9], "rc_basicunit": cfg[10], "rc_qp_min": cfg[11], "rc_qp_max": cfg[12],
                    "fps_num": 1, "fps_den": 15} if cfg in GOLDEN_RC_CONFIGS else {}),
                **({"max_ref_frame": cfg[9]} if cfg in GOLDEN_MRF_CONFIGS else {}),
                **fail,
                "stream_md5": md5(stream), "stream_bytes": len(stream), "slice_qp": slice_qps(stream, qp),
                "recon_md5": [md5(r) for r in rec],
            }
            print(f"{name}: {len(stream)} bytes")
    with open(gpath, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
