"""A/B timing of library builds on bench.py's workload, with the bit-exact
check against the reference MD5s (tests/golden/bench_golden.json).

  python tools/ab_bench.py [lib.so ...]     (default: the in-tree product)

Each build runs in its own process: the driver's configuration (a 5-frame
warm-up call, then 20 frames) and bench.py's default (30, then 120), timed
around the second call.  Development tool.
"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path.insert(0, ROOT)
    import torch

    from hartallo_amd import _lib

    _lib.load_library(os.path.abspath(lib))
    from hartallo_amd import Encoder, synth

    g = json.load(open(os.path.join(ROOT, "tests", "golden", "bench_golden.json")))["bench_1088p_s11"]
    W, H = g["width"], g["height"]
    clip = synth.clip(W, H, 150, 11)
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny = W * H
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + ny // 4) for i in range(150)]
    for warm, steps in ((5, 20), (30, 120)):
        enc = Encoder(W, H, 28, 16, 1, 30)
        if os.environ.get("HL_AB_GEOM"):  # "workgroups,reach,window" or with "/" (hl_amd_set_pipeline)
            enc.set_pipeline(*[int(v) for v in os.environ["HL_AB_GEOM"].replace("/", ",").split(",")])
        enc.set_timing(True)
        outs = [r.annexb() for r in enc.encode_batch_device(ptrs[:warm])]
        torch.cuda.synchronize()
        t = time.perf_counter()
        enc.encode_batch_device(ptrs[warm:warm + steps], collect=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        tm = enc.timing_ms()
        kernel_ms = tm[1]
        outs += [r.annexb() for r in enc.last_batch_results()]
        exact = all(hashlib.md5(o).hexdigest() == m for o, m in zip(outs, g["frame_md5"]))
        hs = enc.last_helper_stats() if hasattr(enc.lib, "hl_amd_last_helper_stats") else "n/a"
        enc.close()
        print(f"{os.path.relpath(lib, ROOT)} geom {os.environ.get('HL_AB_GEOM', 'default')} warmup {warm} steps {steps}: {steps / dt:.2f} fps ({dt * 1e3:.1f} ms, kernel {kernel_ms:.1f} ms, "
              f"records copy {tm[2]:.1f} ms, slice writing {tm[3]:.1f} ms) "
              f"bitexact {exact} helpers {hs}", flush=True)
    # one picture per call (the plugin's per-frame path): P pictures 2..7
    enc = Encoder(W, H, 28, 16, 1, 30)
    outs, ms = [], []
    for i in range(8):
        torch.cuda.synchronize()
        t = time.perf_counter()
        outs.append(enc.encode_device(*ptrs[i]).annexb())
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t) * 1e3)
    exact = all(hashlib.md5(o).hexdigest() == m for o, m in zip(outs, g["frame_md5"]))
    hs = enc.last_helper_stats() if hasattr(enc.lib, "hl_amd_last_helper_stats") else "n/a"
    enc.close()
    print(f"{os.path.relpath(lib, ROOT)} per-picture calls: P pictures {sum(ms[2:]) / 6:.1f} ms each "
          f"({' '.join(f'{m:.1f}' for m in ms)}) bitexact {exact} helpers (last call) {hs}", flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    libs = sys.argv[1:] or [os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so")]
    rc = 0
    for spec in libs:  # lib.so[:VAR=value,...] -- environment of that child
        lib, _, envs = spec.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        if envs:
            print(f"== {lib} with {envs}", flush=True)
        r = subprocess.run([sys.executable, "-u", __file__, "--child", lib], env=env)
        rc = rc or r.returncode
        if r.returncode in (-6, -11, 134, 139):
            break
    sys.exit(rc)


if __name__ == "__main__":
    main()
