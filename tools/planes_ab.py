"""k_planes alone on several library builds (hl_amd_bench_planes: back-to-back
launches on the encoder's reference picture, HIP events), each in its own
process, with the planes checked against the in-tree product's planes of the
same picture.  Development tool, GPU box:

  python tools/planes_ab.py lib1.so [lib2.so ...]
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import torch

    from hartallo_amd import _lib

    _lib.load_library(os.path.abspath(lib))
    from hartallo_amd import Encoder, synth

    W, H = 1920, 1088
    clip = synth.clip(W, H, 2, 11)
    dev = torch.from_numpy(clip).cuda()
    ny = W * H
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(2)]
    enc = Encoder(W, H, 28, 16, 1, 30)
    enc.encode_batch_device(ptrs)
    torch.cuda.synchronize()
    res = {}
    for iters in (50, 200):
        res[iters] = round(1e3 * enc.bench_planes(iters), 2)
    print(json.dumps({"lib": lib, "us_per_launch_50": res[50], "us_per_launch_200": res[200]}), flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    for lib in sys.argv[1:]:
        r = subprocess.run([sys.executable, __file__, "--child", lib], capture_output=True, text=True, timeout=300)
        out = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        print(out[-1] if out else f"{lib}: failed rc={r.returncode} {r.stderr[-500:]}", flush=True)


if __name__ == "__main__":
    main()
