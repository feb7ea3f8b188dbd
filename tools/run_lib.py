"""One pipelined run of the driver's workload on a given library build, for
rocprofv3 passes over builds (tools/pmc_ab.sh): a `warmup`-picture call,
then `steps` pictures in one hl_amd_encode_batch; prints the timing and the
bit-exact check against the reference MD5s.  Development tool.

  python tools/run_lib.py LIB [warmup steps]
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    lib = os.path.abspath(sys.argv[1])
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    import torch

    from hartallo_amd import _lib

    _lib.load_library(lib)
    from hartallo_amd import Encoder, synth

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_golden.json")))["bench_1088p_s11"]
    W, H = g["width"], g["height"]
    clip = synth.clip(W, H, 150, 11)[:warm + steps]
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny = W * H
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(warm + steps)]
    enc = Encoder(W, H, 28, 16, 1, 30)
    enc.set_timing(True)
    outs = [r.annexb() for r in enc.encode_batch_device(ptrs[:warm])]
    torch.cuda.synchronize()
    t = time.perf_counter()
    enc.encode_batch_device(ptrs[warm:], collect=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    outs += [r.annexb() for r in enc.last_batch_results()]
    exact = all(hashlib.md5(o).hexdigest() == m for o, m in zip(outs, g["frame_md5"]))
    print(json.dumps({"lib": os.path.relpath(lib, ROOT), "warmup": warm, "steps": steps, "fps": round(steps / dt, 3),
                      "kernel_ms": round(enc.timing_ms()[1], 2), "bitexact": exact}), flush=True)
    enc.close()


if __name__ == "__main__":
    main()
