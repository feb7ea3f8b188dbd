#!/usr/bin/env python3
"""bench.py -- encoded 1920x1088 frames/s (bit-exact H.264 Baseline), MI355X.

Workload (BASELINE.json configs[2] as the reference can express it, SURVEY
§8(d) c3): 1920x1088 YUV420 IPPP, GOP 30, QP 28, ME range 16, deblocking on,
synthetic input (hartallo_amd.synth, seeded per rank).  A step is one frame
through the whole encode path (quarter-pel planes, MB decisions, deblocking,
CAVLC bitstream); inputs are resident in HBM before the timed region.
The timed frames (by default GOPs 2-5: four IDR pictures and 116 P
pictures, after one warm-up GOP) go through hl_amd_encode_batch: runs of P pictures are
frame-pipelined in one persistent launch (hl_pipeline.h), bit-identical to
encoding them one call at a time (tests/test_gpu_pipeline.py).

Multi-GPU: one independent stream per GPU (frame-sharded throughput mode,
SURVEY §8(e) c5) -- weak scaling, no data-path collective; torch.distributed
(gloo) carries only the barrier and the max-over-ranks of the elapsed time.
Each rank is one independent encoder, as the reference's one hl_codec_t per
stream (hl_codec.c:22-61).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...

Without torchrun (WORLD_SIZE unset) and N > 1, this process only launches N
rank processes (one per GPU, LOCAL_RANK = device) and returns their exit
status; it never touches the GPU itself.  Under torchrun, --gpus must equal
WORLD_SIZE.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

W, H = 1920, 1088
QP, ME_RANGE, DEBLOCK, GOP = 28, 16, 1, 30
BYTES_PER_MB = 2752  # compulsory HBM bytes per macroblock, DESIGN.md / SURVEY §8(d)
# rocprofv3 PMC counters of k_pipeline on this workload (tools/pmc_record.sh:
# SQ issue / wait counters and FETCH_SIZE / WRITE_SIZE, corrected per
# MI355X_MICROARCH.md), summarised per launch of the timed call by
# tools/pmc_summary.py; kept under tools/pmc/ (travels to the GPU box; a copy
# in profiles/).  They describe the library whose SHA-256 they name.
PMC_FILE = os.path.join(ROOT, "tools", "pmc", "pmc_k_pipeline.json")
STAT_KEYS = ("runs", "per_picture", "fallbacks", "waits_gave_up", "chain_walks")
MAX_RUN = 128  # pictures per pipelined launch (kMaxRun, hl_encoder.hip)
# The synthetic stream is always generated for BENCH_CLIP_FRAMES frames (its
# texture depends on the clip length) and its first warmup + steps frames are
# encoded; tests/golden/bench_golden.json holds the reference encoder's
# per-frame output MD5s for it (tests/golden/make_bench_golden.py), checked
# after the timed region.
BENCH_CLIP_FRAMES = 150
BENCH_GOLDEN = os.path.join(ROOT, "tests", "golden", "bench_golden.json")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
SHADER_CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)
PLANES_PAD = 40  # kPad of the quarter-pel planes (hl_mbcore.h)


def load_pmc(lib_path, warmup, steps, workgroups, streams_per_gpu):
    """The recorded counters when they were taken on this exact library (the
    file that was loaded) and workload -- picture size, warm-up and timed
    pictures, k_pipeline workgroups, streams sharing the GPU -- else (None,
    why not)."""
    import hashlib

    from hartallo_amd import _lib

    if not os.path.exists(PMC_FILE):
        return None, "no counters recorded (tools/pmc_record.sh)"
    if not lib_path or not os.path.exists(lib_path):
        return None, "library not found"
    pmc = json.load(open(PMC_FILE))
    sha = hashlib.sha256(open(lib_path, "rb").read()).hexdigest()
    # the same library file, or one whose code (device and host sections) is
    # the same: a relink can reorder the ELF string tables only
    code = _lib.code_sha256(lib_path) if pmc.get("code_sha256") else None
    if pmc.get("lib_sha256") != sha and (code is None or pmc.get("code_sha256") != code):
        return None, f"stale: recorded on library {pmc.get('lib_sha256', '?')[:12]}, this one is {sha[:12]} (rerun tools/pmc_record.sh)"
    want = {"warmup": warmup, "steps": steps, "width": W, "height": H, "workgroups": workgroups, "streams_per_gpu": streams_per_gpu}
    diff = {k: (pmc.get(k), v) for k, v in want.items() if pmc.get(k) != v}
    if diff:
        return None, "recorded on another workload: " + ", ".join(f"{k} {a} (here {b})" for k, (a, b) in diff.items())
    same = "library" if pmc.get("lib_sha256") == sha else "code"
    return pmc, f"tools/pmc/pmc_k_pipeline.json, {same} sha256 {(sha if same == 'library' else code)[:12]}, recorded {pmc.get('recorded', '?')}"


def critical_path_steps(frames, mbw, mbh, reach=2):
    """Longest dependency chain of a pipelined run of `frames` pictures, in
    macroblock tasks (hl_pipeline.h task_deps: (x-1, y), (x+1, y-1) -- (x,
    y-1) in the last column -- and picture f-1's reach_task(x+R, y+R)): the
    run's time per step of it is the macroblock latency its critical path
    achieved."""
    import numpy as np

    prev = None
    for _ in range(frames):
        d = np.zeros((mbh, mbw), dtype=np.int64)
        for y in range(mbh):
            for x in range(mbw):
                v = 0
                if x > 0:
                    v = d[y, x - 1]
                if y > 0:
                    v = max(v, d[y - 1, min(x + 1, mbw - 1)])
                if prev is not None:
                    ty = min(y + reach + 2, mbh - 1)
                    tx = min(x + reach + (3 if ty == mbh - 1 else 2), mbw - 1)
                    v = max(v, prev[ty, tx])
                d[y, x] = v + 1
        prev = d
    return int(prev.max())


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _ref_encoders():
    """The reference encoder builds a CPU baseline can time, best first: its
    x86-intrinsic build (oracle/_ref/ref_enc_sse, the encoder BASELINE.json's
    north star names), its pure-C build (oracle/_ref/ref_enc), else the
    bit-exact C restatement (oracle/)."""
    cands = [(os.path.join(ROOT, "oracle", "_ref", "ref_enc_sse"), "reference",
              "x86-intrinsic (SSE2-SSE4.2) build of the reference sources (hl_codec_264_deblock.c keeps its C path: its "
              "SSE header declares the threshold table const, which gcc rejects, oracle/Makefile)"),
             (os.path.join(ROOT, "oracle", "_ref", "ref_enc"), "reference", "pure-C build of the reference sources"),
             (os.path.join(ROOT, "oracle", "_build", "hlenc_oracle"), "port", "bit-exact C restatement (oracle/hl_oracle.c)")]
    return [c for c in cands if os.path.exists(c[0])]


def _timed_mix(first, steps):
    """IDR and P pictures among the timed frames [first, first + steps)."""
    n_i = sum(1 for f in range(first, first + steps) if f % GOP == 0)
    return n_i, steps - n_i


def cpu_baseline(frames_host, n_frames, first, steps, parallel=8):
    """Times the reference encoder on the first n_frames of this rank's
    workload (1 I + n_frames-1 P pictures), encode time only, and weights
    its measured I- and P-picture times to the timed frames' mix (the
    driver's --warmup 5 --steps 20 times P pictures only).  Then the same
    sample on `parallel` processes at once (one per core, SURVEY §6's
    N-process figure): their summed rate."""
    found = _ref_encoders()
    if not found:
        return None
    exe, kind, what = found[0]
    n_i, n_p = _timed_mix(first, steps)

    def rate(info):
        t_p = info["p_seconds"] / (n_frames - 1)
        t_i = info["seconds"] - info["p_seconds"]
        return steps / (n_i * t_i + n_p * t_p), t_i, t_p

    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "in.yuv")
        frames_host[:n_frames].tofile(inp)

        def cmd(k):
            return [exe, str(W), str(H), str(n_frames), str(QP), str(ME_RANGE), str(DEBLOCK), str(GOP), "0", inp,
                    os.path.join(td, f"o{k}"), "quiet"]

        r = subprocess.run(cmd(0), capture_output=True, text=True, check=True)
        fps1, t_i, t_p = rate(json.loads(r.stdout.strip().splitlines()[-1]))
        try:
            cores = len(os.sched_getaffinity(0))
        except AttributeError:
            cores = os.cpu_count() or 1
        npar = max(1, min(parallel, cores))
        procs = [subprocess.Popen(cmd(k + 1), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for k in range(npar)]
        outs = [p.communicate() for p in procs]
        if any(p.returncode for p in procs):
            par = None
        else:
            rates = [rate(json.loads(o[0].strip().splitlines()[-1]))[0] for o in outs]
            par = {"value": round(sum(rates), 4), "unit": "frames/s", "cores": npar, "kind": kind,
                   "sample": f"{npar} processes of the same build at once, each on the same sample, summed rates "
                             f"(per process {min(rates):.4f}-{max(rates):.4f} frames/s)"}
    return {
        "value": round(fps1, 4),
        "unit": "frames/s",
        "cores": 1,
        "kind": kind,
        "sample": f"{what}, first {n_frames} frames (1 I + {n_frames - 1} P) of the same 1920x1088 QP{QP} stream, encode time only, "
                  f"1 thread on {cpu_model()}: I picture {t_i:.2f} s, P pictures {t_p:.2f} s each, weighted to the timed "
                  f"frames ({n_i} I + {n_p} P)",
        "parallel": par,
    }


def svc_cpu_baseline(clips, g, n_aus, first, steps):
    """Times the reference encoder as an SVC encoder (the reference sources
    through hl_codec_add_layer + hl_codec_encode: oracle/_ref/ref_svc_sse,
    its x86-intrinsic build, else ref_svc, the pure-C one) on the first n_aus
    access units of the config-4 stream, single thread, weighted to the timed
    access units' I/P mix."""
    cands = [(os.path.join(ROOT, "oracle", "_ref", "ref_svc_sse"), "x86-intrinsic (SSE2-SSE4.2) build"),
             (os.path.join(ROOT, "oracle", "_ref", "ref_svc"), "pure-C build")]
    found = [c for c in cands if os.path.exists(c[0])]
    if not found or n_aus < 2:
        return None
    exe, what = found[0]
    L = g["layers"]
    with tempfile.TemporaryDirectory() as td:
        ins = []
        for l in range(L):
            ins.append(os.path.join(td, f"in{l}.yuv"))
            clips[l][:n_aus].tofile(ins[-1])
        cmd = [exe, str(L), str(g["w0"]), str(g["h0"]), str(n_aus), str(g["qp"]), str(g["me_range"]), str(g["deblock"]), str(g["gop"]),
               str(g["early_term"]), os.path.join(td, "o")] + ins + ["quiet"]
        r = subprocess.run(cmd, capture_output=True, text=True, check=True)
        info = json.loads(r.stdout.strip().splitlines()[-1])
    t_p = info["p_seconds"] / (n_aus - 1)
    t_i = info["seconds"] - info["p_seconds"]
    n_i = sum(1 for f in range(first, first + steps) if f % g["gop"] == 0)
    n_p = steps - n_i
    return {
        "value": round(steps / (n_i * t_i + n_p * t_p), 4),
        "unit": "access units/s",
        "cores": 1,
        "kind": "reference",
        "sample": f"{what} of the reference sources as an SVC encoder ({os.path.basename(exe)}), first {n_aus} access units "
                  f"(1 I + {n_aus - 1} P) of the same 3-layer stream, encode time only, 1 thread on {cpu_model()}: I access unit "
                  f"{t_i:.2f} s, P access units {t_p:.2f} s each, weighted to the timed access units ({n_i} I + {n_p} P)",
    }


def check_bitexact(outputs, seed):
    """True / False when every frame's Annex-B output matches the reference
    encoder's MD5 for this stream (tests/golden/bench_golden.json), None when
    no reference MD5s cover it."""
    import hashlib

    key = f"bench_1088p_s{seed}"
    if not os.path.exists(BENCH_GOLDEN):
        return None
    gold = json.load(open(BENCH_GOLDEN)).get(key)
    if not gold or len(outputs) > len(gold["frame_md5"]) or gold["width"] != W or gold["height"] != H or gold["qp"] != QP:
        return None
    return all(hashlib.md5(o).hexdigest() == g for o, g in zip(outputs, gold["frame_md5"]))


SVC_WORKLOAD = "c4_svc3_480x272_s41"  # tests/golden/svc_golden.json (make_svc_golden.py)
SVC_GOLDEN = os.path.join(ROOT, "tests", "golden", "svc_golden.json")


def run_svc(args):
    """BASELINE config 4: 3 dyadic spatial layers 480x272 / 960x544 /
    1920x1088 (the reference's layer ratios must be powers of two,
    hl_codec.c:113-121), IPPP GOP 30, QP 28, ME 16, deblocking.  A step is
    one access unit (all layers of one frame).  One GPU codes every layer
    (hl_amd_encode_layers_batch: the enhancement layers of an access unit
    overlap the base run's later pictures).  With N ranks each rank codes a
    whole stream (HL_SVC_SHARD=streams, the default: no data-path exchange,
    weak scaling), or the layers are sharded over ranks (HL_SVC_SHARD=layers,
    hartallo_amd/svc_pipeline.py: the base layer on one rank, the
    enhancement layers on the next, the layer state handed over by
    point-to-point sends -- RCCL over xGMI; lower latency per access unit,
    lower throughput).  The reference
    encoder's per-access-unit MD5s cover 31 access units (the timed ones and
    the warm-up), checked after the timed region."""
    import hashlib

    import torch

    from hartallo_amd import SvcEncoder, dist, svc_pipeline, synth

    g = json.load(open(SVC_GOLDEN))[SVC_WORKLOAD]
    L, w0, h0 = g["layers"], g["w0"], g["h0"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # ranks beyond the visible GPUs share them (gloo rehearsals on a one-GPU box)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    nccl = world > 1 and os.environ.get("HL_SVC_BACKEND", "nccl") == "nccl"
    if world > 1:
        import torch.distributed as tdist

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        tdist.init_process_group("nccl" if nccl else "gloo", rank=rank, world_size=world,
                                 **({"device_id": torch.device(f"cuda:{local}")} if nccl else {}))
    shard = os.environ.get("HL_SVC_SHARD", "streams")
    if shard not in ("streams", "layers"):
        raise SystemExit(f"HL_SVC_SHARD={shard}: expected streams or layers")
    streams = world == 1 or shard == "streams"
    if streams:  # every rank codes every layer of its own stream
        role = svc_pipeline.Role(rank, 0, 1, 0, L - 1, -1, -1, rank)
    else:
        role = svc_pipeline.role_of(rank, world, L)
    n = min(args.warmup + args.steps, g["frames"])
    steps = n - args.warmup
    clips = synth.svc_clips(w0 << (L - 1), h0 << (L - 1), L, g["frames"], g["seed"])
    planes = []
    for l in range(L):
        w, h = w0 << l, h0 << l
        dev = torch.from_numpy(clips[l][:n]).to(f"cuda:{local}")
        planes.append([(dev[i, :w * h], dev[i, w * h:w * h * 5 // 4], dev[i, w * h * 5 // 4:]) for i in range(n)])
    torch.cuda.synchronize()
    enc = SvcEncoder(w0, h0, L, g["qp"], g["me_range"], g["deblock"], g["gop"], g["early_term"], local, role.first, role.last)
    enc.set_timing(True)
    ad = svc_pipeline.GpuLayerAdapter(enc, planes)
    if nccl:
        mk = lambda nb: torch.empty(nb, dtype=torch.uint8, device=f"cuda:{local}")  # noqa: E731
    else:
        # gloo moves host tensors: stage the layer state through host memory
        class _Host:
            def __init__(self, a):
                self.a = a

            def __getattr__(self, k):
                return getattr(self.a, k)

            def export_layer(self, layer, buf):
                d = torch.empty(buf.numel(), dtype=torch.uint8, device=f"cuda:{local}")
                self.a.export_layer(layer, d)
                buf.copy_(d.cpu())

            def import_layer(self, layer, buf):
                self.a.import_layer(layer, buf.to(f"cuda:{local}"))
        ad = _Host(ad)
        mk = lambda nb: torch.empty(nb, dtype=torch.uint8)  # noqa: E731
    tdist = None
    if world > 1:
        import torch.distributed as tdist

    class _Split:  # warm-up access units, then the timed ones, through one pipeline state
        def __init__(self, a, off):
            self.a, self.off = a, off

        def __getattr__(self, k):
            return getattr(self.a, k)

        def encode(self, layer, t):
            return self.a.encode(layer, t + self.off)

    if streams:
        # every layer on this GPU: hl_amd_encode_layers_batch (the base-layer
        # pictures frame-pipelined; an access unit's enhancement layers while
        # the run codes the next base pictures)
        ptrs = [[tuple(p.data_ptr() for p in planes[l][i]) for i in range(n)] for l in range(L)]

        def batch(lo, hi):
            return [(r.hdr, r.data) for r in enc.encode_layers_batch_device([p[lo:hi] for p in ptrs])]

        parts = batch(0, args.warmup) if args.warmup else []
        torch.cuda.synchronize()
        if tdist:
            tdist.barrier()
        t0 = time.perf_counter()
        parts += batch(args.warmup, n)
    else:
        parts = svc_pipeline.run_access_units(ad, role, None, args.warmup, tdist, mk) if args.warmup else []
        tdist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        parts += svc_pipeline.run_access_units(_Split(ad, args.warmup), role, None, steps, tdist, mk)
    torch.cuda.synchronize()
    if tdist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    if tdist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        if nccl:
            t = t.cuda()
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())
        allp = [None] * world
        tdist.all_gather_object(allp, parts)
    else:
        allp = [parts]
    if streams:
        groups = list(range(world))
        member_of = {r: [r] for r in groups}
    else:
        groups = sorted({svc_pipeline.role_of(r, world, L).group for r in range(world)})
        member_of = {gi: [r for r in range(world) if svc_pipeline.role_of(r, world, L).group == gi] for gi in groups}
    ok = True
    for gi in groups:
        members = member_of[gi]
        aus = svc_pipeline.assemble([allp[r] for r in members])
        ok = ok and [hashlib.md5(a).hexdigest() for a in aus] == g["au_md5"][:n]
    roofline = base = None
    if rank == 0 and streams:
        # dominant kernel: k_pipeline of the base run (one launch per batch);
        # algorithmic bytes = 2752 B per base MB x MBs per launch
        ms = enc.timing_ms()
        if enc.last_mb_launches() == 1 and ms[1] > 0:
            nmb0 = (w0 // 16) * (h0 // 16)
            ach = BYTES_PER_MB * nmb0 * steps / (ms[1] / 1e3) / 1e9
            roofline = {"bound": "hbm", "achieved": round(ach, 4), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                        "traffic": None, "kernel": "k_pipeline (base layer run)", "avg_launch_us": round(ms[1] * 1e3, 2),
                        "frames_per_launch": steps,
                        "note": "latency-bound MB wavefront of the 480x272 base layer; the enhancement layers run beside it"}
        if world == 1 and not args.no_cpu_baseline:
            base = svc_cpu_baseline(clips, g, min(args.cpu_frames, n), args.warmup, steps)
    if rank == 0:
        total = len(groups) * steps
        print(json.dumps({
            "metric": "SVC 3-layer (480x272/960x544/1920x1088) access units/sec (bit-exact)",
            "value": round(total / elapsed, 4), "unit": "access units/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8/int32", "data": "synthetic (hartallo_amd.synth.svc_clips, seed 41)",
            "config": {"workload": "BASELINE config 4: dyadic spatial SVC, 3 layers, IPPP GOP30 QP28 ME16 deblock",
                       "layers": [[w0 << l, h0 << l] for l in range(L)], "streams": len(groups),
                       "parallelism": ("all layers on one GPU per stream, base layer frame-pipelined, enhancement layers "
                                       "overlapping the base run") if streams else "layer-sharded",
                       "exchange": ("rccl" if nccl else "gloo-host") if not streams else None},
            "bitexact": ok,
            "bitexact_check": "every access unit (warm-up and timed) of every stream vs the reference encoder's per-AU MD5s "
                              "(tests/golden/svc_golden.json, oracle/_ref/ref_svc)",
            "rank0_layers": [role.first, role.last],
            # batch path: [1] = the base run's k_pipeline launch (HIP events); per access unit: the base picture's run
            "rank0_last_batch_ms": {"base_run_device": round(enc.timing_ms()[1], 3) if role.first == 0 else None,
                                    "last_au_enhancement_layers_device": round(enc.layer_ms(), 3)},
            "roofline": roofline,
            "cpu_baseline": base,
        }), flush=True)
    enc.close()
    if tdist:
        tdist.destroy_process_group()


def spawn_ranks(n, argv, script=None):
    """Runs this script as n rank processes (RANK = LOCAL_RANK = r,
    WORLD_SIZE = LOCAL_WORLD_SIZE = n, a free rendezvous port on 127.0.0.1)
    and returns the first non-zero exit status, else 0.  The caller has not
    touched the GPU and does not afterwards: it only launches and waits.
    Ranks inherit stdout/stderr (rank 0 prints the line).  When one rank
    fails the others are terminated: they would wait forever at the next
    collective.  Deadlines: HL_BENCH_TIMEOUT seconds for the whole group
    (default 1800), and HL_BENCH_GRACE seconds (default 120) for the others
    once any rank has exited, even with 0 (a peer stuck at a collective or
    on the GPU would otherwise be waited for forever); stragglers get
    SIGTERM, then SIGKILL 10 s later, and the status is non-zero.  A failed
    rendezvous is not retried on another port: a rank that failed may have
    failed on the GPU, and GPU steps are never retried."""
    import signal
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HL_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env))
    rc = 0
    live = list(procs)
    t0 = time.monotonic()
    deadline = t0 + float(os.environ.get("HL_BENCH_TIMEOUT", "1800"))
    grace = float(os.environ.get("HL_BENCH_GRACE", "120"))
    term_at = None  # when the stragglers were sent SIGTERM

    def stop(why):
        nonlocal term_at
        if term_at is None:
            print(f"bench.py: {why}; stopping ranks {[procs.index(q) for q in live]}", file=sys.stderr, flush=True)
            for q in live:
                q.send_signal(signal.SIGTERM)
            term_at = time.monotonic()

    try:
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c and not rc:
                    rc = c if c > 0 else 128 - c
                    stop(f"rank {procs.index(p)} exited with status {c}")
                elif live and deadline > time.monotonic() + grace:
                    deadline = time.monotonic() + grace  # the others have `grace` seconds to follow
            now = time.monotonic()
            if live and term_at is None and now > deadline:
                rc = rc or 124
                stop(f"deadline reached after {now - t0:.0f} s")
            if live and term_at is not None and now > term_at + 10:
                for q in live:
                    q.kill()
                for q in live:
                    q.wait()
                live = []
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in live:
            p.send_signal(signal.SIGTERM)
        raise
    return rc


def resolve_world(gpus):
    """(world, launch): the number of ranks and whether this process must
    launch them.  WORLD_SIZE set (torchrun, or spawn_ranks) fixes the world;
    an explicit --gpus that disagrees with it is an error, not a silent
    one-GPU run."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None:
        world = int(env)
        if gpus is not None and gpus != world:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch {gpus} ranks "
                             f"(torchrun --nproc-per-node {gpus}) or run without torchrun")
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}: need at least one GPU")
    return n, n > 1


def rank_devices(local):
    """[(rank, device index, PCI bus id)] of every rank, gathered on every
    rank (gloo), so the line shows which physical GPUs ran."""
    import torch
    import torch.distributed as tdist

    p = torch.cuda.get_device_properties(local)
    mine = {"rank": tdist.get_rank() if tdist.is_initialized() else 0, "device": local,
            "pci_bus_id": f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                          f"{getattr(p, 'pci_device_id', 0):02x}"}
    if not tdist.is_initialized():
        return [mine]
    allr = [None] * tdist.get_world_size()
    tdist.all_gather_object(allr, mine)
    return allr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks, one per GPU (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=4 * GOP)  # four whole GOPs (IDR + 29 P pictures each), one pipelined launch
    ap.add_argument("--warmup", type=int, default=GOP)  # the first GOP (also warms the pipelined path)
    ap.add_argument("--cpu-frames", type=int, default=6)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--streams", type=int, default=1, help="streams per process, in shared pipelined runs (hl_amd_encode_streams)")
    ap.add_argument("--svc", action="store_true", help="BASELINE config 4 (spatial SVC) instead of the headline workload")
    args = ap.parse_args()
    world_req, launch = resolve_world(args.gpus)
    if launch:  # before anything imports torch or touches a GPU
        sys.exit(spawn_ranks(world_req, sys.argv[1:]))
    if args.svc:
        if "--steps" not in sys.argv:
            args.steps = 30
        if "--warmup" not in sys.argv:
            args.warmup = 1
        return run_svc(args)

    import torch

    from hartallo_amd import Encoder, dist, synth

    rank, world, local = dist.init_from_env()
    if world != world_req:
        raise SystemExit(f"bench.py: process group of {world} ranks, expected {world_req}")
    local %= max(1, torch.cuda.device_count())  # ranks beyond the visible GPUs share them (rehearsals on a one-GPU box)
    torch.cuda.set_device(local)
    ranks = rank_devices(local)
    pg_world = dist.world_size()

    n_frames = args.warmup + args.steps
    K = max(1, args.streams)  # streams this process encodes (one encoder each, shared pipelined runs)
    seeds = [dist.stream_seed(rank * K + si) for si in range(K)]
    frames_host = [synth.clip(W, H, max(n_frames, BENCH_CLIP_FRAMES), sd)[:n_frames] for sd in seeds]
    # inputs resident in HBM before timing
    devs = [torch.from_numpy(fh).to(f"cuda:{local}") for fh in frames_host]
    torch.cuda.synchronize()
    ny, nc = W * H, W * H // 4
    ptrs = [[(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + nc) for i in range(n_frames)] for dev in devs]

    encs = [Encoder(W, H, QP, ME_RANGE, DEBLOCK, GOP, 0, local) for _ in range(K)]
    enc = encs[0]  # launches the shared runs (its diagnostics describe them)
    # streams sharing one GPU (more ranks on this node than visible GPUs):
    # each rank's persistent run takes its share of the CUs, so the runs
    # execute side by side instead of taking turns for the whole device
    # (several streams per GPU fill the MB wavefront's ramp and
    # tail).  More than two processes per GPU time-slice the device (4 of
    # them collapsed to 3.5 frames/s, profiles/r03_streams_sharing_hw_queues.log):
    # several streams per GPU belong in one process (--streams).
    share = -(-int(os.environ.get("LOCAL_WORLD_SIZE", "1")) // max(1, torch.cuda.device_count()))
    warning = None
    if share > 2:
        warning = (f"{share} processes share each GPU: the device time-slices between processes and persistent runs stall "
                   "each other's dependency waits; run several streams in one process instead (--streams)")
        if rank == 0:
            print(f"bench.py: warning: {warning}", file=sys.stderr, flush=True)
    wg_used = 0  # k_pipeline workgroups (0: one per resident slot)
    if share > 1:
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        wg_used = max(1, cus // share)
        enc.set_pipeline(wg_used, 2, 64)

    def encode(lo, hi, collect):
        if K == 1:
            return [enc.encode_batch_device(ptrs[0][lo:hi], collect=collect)]
        return Encoder.encode_streams_device(encs, [p[lo:hi] for p in ptrs], collect=collect)

    def stats_sum():  # the launches (encoder 0) and every stream's per-picture path
        st = [e.last_batch_stats() for e in encs]
        return {k: st[0][k] if k in ("runs", "chain_walks", "waits_gave_up") else sum(x[k] for x in st) for k in STAT_KEYS}

    outputs = [[] for _ in range(K)]
    warm = {k: 0 for k in STAT_KEYS}
    if args.warmup:  # same entry point as the timed frames (warms the pipelined path and its buffers)
        for si, rs in enumerate(encode(0, args.warmup, True)):
            outputs[si] += [r.annexb() for r in rs]
        warm = stats_sum()
    enc.set_timing(True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out_bytes = sum(encode(args.warmup, n_frames, False))
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = dist.max_over_ranks(time.perf_counter() - t0)
    ms = enc.timing_ms()
    mb_ms, mb_launches = ms[1], enc.last_mb_launches()  # the (last) pipelined launch
    stats = stats_sum()
    # how every rank's calls ran (fallbacks to the per-picture path would show here), summed over ranks
    tot = dist.sum_over_ranks([stats[k] for k in STAT_KEYS] + [warm["fallbacks"] + warm["waits_gave_up"] + warm["per_picture"]])
    pipeline = dict(zip(STAT_KEYS, tot[:len(STAT_KEYS)]))
    pipeline["warmup_off_pipeline"] = tot[-1]
    pipeline["scope"] = ("timed call (hl_amd_last_batch_stats), summed over ranks (runs: launches); warmup_off_pipeline = "
                         "warm-up pictures not coded by a clean run")
    # bit-exactness of everything this rank encoded, outside the timed region
    bitexact = True
    for si, e in enumerate(encs):
        outputs[si] += [r.annexb() for r in e.last_batch_results()]
        b = check_bitexact(outputs[si], seeds[si])
        bitexact = None if b is None or bitexact is None else (bitexact and b)
    # every rank joins the collective (-1: no reference MD5s cover this rank's streams)
    ex = dist.min_over_ranks(-1 if bitexact is None else (1 if bitexact else 0))
    bitexact_all = None if ex < 0 else ex
    # pictures of the last pipelined launch (per stream): runs span GOPs, up to MAX_RUN pictures each
    run_frames = (args.steps - 1) % MAX_RUN + 1 if mb_launches == 1 else 1

    # the HBM-bound kernel of the path on its own: quarter-pel planes of a
    # 1088p reference, read 1 B/px + write 4 B per padded pixel
    planes_ms = enc.bench_planes(50)
    pw, ph = W + 2 * PLANES_PAD, H + 2 * PLANES_PAD
    planes_bytes = W * H + 4 * pw * ph

    base = None
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region, on rank 0 only
        base = cpu_baseline(frames_host[0], min(args.cpu_frames, n_frames), args.warmup, args.steps)

    if rank == 0:
        total = world * K * args.steps
        fps = total / elapsed
        nmb = (W // 16) * (H // 16)
        # dominant kernel: k_pipeline (one launch per run of pictures);
        # algorithmic bytes per launch = 2752 B x MBs per launch
        avg_launch_s = (mb_ms / 1e3) / mb_launches
        bytes_per_launch = BYTES_PER_MB * nmb * run_frames * K / mb_launches
        achieved = bytes_per_launch / avg_launch_s / 1e9
        from hartallo_amd import _lib

        pmc, pmc_note = load_pmc(getattr(_lib, "LOADED_PATH", None) or _lib.LIB_PATH, args.warmup, args.steps, wg_used, share * K)
        # the achieved macroblock latency along the run's critical path, and
        # VALU issue against one wave64 VALU instruction per SIMD per cycle
        cp_steps = critical_path_steps(run_frames, W // 16, H // 16) if mb_launches == 1 else None
        cp_us = round(avg_launch_s * 1e6 / cp_steps, 2) if cp_steps else None
        cus = torch.cuda.get_device_properties(local).multi_processor_count
        valu_util = (round(pmc["valu_insts_per_mb"] * nmb * run_frames * K / avg_launch_s / (4 * cus * SHADER_CLOCK_HZ), 4)
                     if pmc and mb_launches == 1 else None)
        line = {
            "metric": "1080p encoded frames/sec (bit-exact) at 1/2/4/8 MI355X; macroblocks/sec/GPU",
            "value": round(fps, 4),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/int32",
            "data": "synthetic (hartallo_amd.synth, seeded per rank)",
            "config": {"workload": "1920x1088 YUV420 IPPP GOP30 QP28 ME16 deblock, one stream per GPU, frame-pipelined", "width": W, "height": H,
                       "qp": QP, "me_range": ME_RANGE, "deblock": DEBLOCK, "gop": GOP, "parallelism": f"streams{world * K}",
                       "streams_per_gpu": share * K, "streams_per_process": K},
            "mb_per_s_per_gpu": round(fps / world * share * nmb, 1),
            # which physical GPUs ran: the process group's size and every rank's device
            "process_group_world_size": pg_world,
            "ranks": ranks,
            "distinct_gpus": len({r["pci_bus_id"] for r in ranks}),
            "warning": warning,
            "bitexact": bitexact_all if bitexact_all is None else bool(bitexact_all),
            "bitexact_check": "every frame of every rank (warm-up and timed) vs the reference encoder's per-frame MD5s "
                              "(tests/golden/bench_golden.json, oracle/_ref/ref_enc on the same synthetic stream)",
            "pipeline": pipeline,
            "bitstream_bytes_per_frame": round(out_bytes / args.steps, 1),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": round(pmc["traffic_bytes_per_mb"] * nmb * run_frames * K) if pmc and mb_launches == 1 else None,
                         "kernel": "k_pipeline", "avg_launch_us": round(avg_launch_s * 1e6, 2),
                         "frames_per_launch": run_frames,
                         "note": "latency-bound MB wavefront, frames pipelined; achieved = 2752 B/MB x MBs per launch / launch time",
                         # what bounds it instead (rocprofv3 SQ counters of this library on this workload, tools/pmc_record.sh)
                         "sq_wait_frac": pmc["sq_wait_frac"] if pmc else None,
                         "sq_issue_frac": pmc["sq_issue_frac"] if pmc else None,
                         "valu_insts_per_mb": pmc["valu_insts_per_mb"] if pmc else None,
                         "valu_util": valu_util,
                         "valu_util_def": "VALU wave-instructions/s / (4 SIMD x CUs x 2.4 GHz)",
                         "critical_path_steps": cp_steps,
                         "critical_path_us_per_step": cp_us,
                         "pmc": pmc_note},
            "planes_roofline": {"kernel": "k_planes", "bound": "hbm", "achieved": round(planes_bytes / (planes_ms / 1e3) / 1e9, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(planes_bytes / (planes_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": planes_bytes, "avg_launch_us": round(planes_ms * 1e3, 2),
                                "note": "50 back-to-back launches on the reference picture, HIP events on the encoder's stream"},
            "cpu_baseline": base,
        }
        print(json.dumps(line), flush=True)
    for e in encs:
        e.close()
    dist.shutdown()


if __name__ == "__main__":
    main()
