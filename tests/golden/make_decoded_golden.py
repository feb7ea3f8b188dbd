"""Per-frame MD5s of the reference *decoder's* output for the reference
encoder's own streams (the conformance gate, tests/test_conformance.py).

oracle/_ref/ref_dec (the reference's decoder, built by oracle/Makefile from
its sources) decodes:
  * every committed golden stream tests/golden/<name>.264 -> golden.json
    [name]["decoded_md5"] (or ["decoder_failure"] when the reference decoder
    does not decode that stream: it crashes, drops pictures or returns
    pictures of another size -- recorded, not hidden);
  * the reference encoder's stream (oracle/_ref/ref_enc) of the first
    DECODED_FRAMES[name] frames of the BASELINE-sized workloads of
    bench_golden.json -> bench_golden.json[name]["decoded_md5"].

Run in the build container (needs oracle/_ref/ref_enc and ref_dec):
  python tests/golden/make_decoded_golden.py
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

from hartallo_amd import synth  # noqa: E402

REF_ENC = os.path.join(ROOT, "oracle", "_ref", "ref_enc")
REF_DEC = os.path.join(ROOT, "oracle", "_ref", "ref_dec")
DECODED_FRAMES = {"c2_720p_s7": 31, "bench_1088p_s11": 25}


def decode(stream_path, w, h, n):
    """Per-frame MD5s of the decoded pictures, or (None, reason)."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "d.yuv")
        r = subprocess.run([REF_DEC, stream_path, out], capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            return None, f"ref_dec exit status {r.returncode}"
        data = open(out, "rb").read()
    fs = w * h * 3 // 2
    if len(data) != n * fs:
        return None, f"decoded {len(data)} bytes, expected {n} pictures of {fs}"
    return [hashlib.md5(data[i * fs:(i + 1) * fs]).hexdigest() for i in range(n)], None


def small(name, g):
    # (a reference-failure golden holds the pictures before its failing frame)
    md5s, why = decode(os.path.join(HERE, name + ".264"), g["width"], g["height"], g.get("fail_frame", g["frames"]))
    return name, md5s, why


def bench(name, g):
    n = DECODED_FRAMES[name]
    w, h = g["width"], g["height"]
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.yuv")
        synth.clip(w, h, g["frames"], g["seed"])[:n].tofile(inp)  # the workload's clip, first n frames
        pre = os.path.join(td, "o")
        subprocess.run([REF_ENC, str(w), str(h), str(n), str(g["qp"]), str(g["me_range"]), str(g["deblock"]), str(g["gop"]), "0",
                        inp, pre, "quiet"], check=True, capture_output=True)
        md5s, why = decode(pre + ".264", w, h, n)
    return name, md5s, why


def main():
    for tool in (REF_ENC, REF_DEC):
        if not os.path.exists(tool):
            sys.exit(f"{tool} missing: run `make -C oracle ref` where /root/reference exists")
    gpath, bpath = os.path.join(HERE, "golden.json"), os.path.join(HERE, "bench_golden.json")
    gold, bgold = json.load(open(gpath)), json.load(open(bpath))
    only = set(sys.argv[1:])  # names: only those entries are (re)made
    with ThreadPoolExecutor(max_workers=8) as ex:
        jobs = ([ex.submit(small, k, v) for k, v in gold.items() if not only or k in only] +
                [ex.submit(bench, k, bgold[k]) for k in DECODED_FRAMES if not only or k in only])
        for j in jobs:
            name, md5s, why = j.result()
            table = gold if name in gold else bgold
            table[name].pop("decoded_md5", None)
            table[name].pop("decoder_failure", None)
            if md5s is None:
                table[name]["decoder_failure"] = why
            else:
                table[name]["decoded_md5"] = md5s
            print(name, why or f"{len(md5s)} pictures", flush=True)
    for path, table in ((gpath, gold), (bpath, bgold)):
        with open(path, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
