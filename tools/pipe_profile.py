"""Where the workgroups of a pipelined run spend their time (profiling build,
`make profile`).

  python tools/pipe_profile.py [frames] [workgroups,R,window]

Development tool: 1920x1088 QP28 ME16 deblock; I and P warm-up pictures one
call at a time, then `frames` P pictures in one hl_amd_encode_batch.  Prints
the per-workgroup split of k_pipeline's lifetime (task-start waits,
decisions, deblocking + planes, the rest = taking tasks / draining) and the
per-MB phases of the decisions.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from hartallo_amd import _lib  # noqa: E402

_lib.load_library(os.environ.get("HL_LIB") or os.path.join(ROOT, "build", "prof", "hartallo_amd", "libhartallo_amd.so"))
from hartallo_amd import Encoder, synth  # noqa: E402

PHASES = ["eval:block", "eval:nC", "eval:reduce", "search_partition", "mvp", "guess_intra(P)", "mb_begin", "mb_end", "whole MB",
          "reach_wait", "intra:i16", "intra:i4", "early-term modes", "inter finalize", "", "", "step:candidates", "step:selection", "", "helper join"]
PHASES[14], PHASES[15], PHASES[18] = "reconstruct_chroma", "intra tail (chroma, CBP)", "inter_pred_mb"  # default profiling build
if os.environ.get("HL_BAR_NAMES"):  # a build with -DHL_BAR_PROF: barrier cycles per MB (all waves / most / least waiting wave)
    PHASES[14] = "barriers:all waves"
    PHASES[15] = "barriers:max wave"
    PHASES[18] = "barriers:min wave"
if os.environ.get("HL_I4_NAMES"):  # a build with -DHL_I4_PROF: slots 12..15 time guess_i4's wavefront steps
    PHASES[12:16] = ["i4:neighbours+nC", "i4:modes", "i4:step barrier", "i4:resolution"]
if os.environ.get("HL_STEP_NAMES"):  # a build with -DHL_STEP_PROF: slots 12..15, 18, 19 time the steps' sub-phases
    PHASES[12:16] = ["step:loads", "step:quad work", "step:eval barrier", "step:results+minima"]
    PHASES[18] = "step:chain resolved"
    PHASES[19] = "step:cands generated"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    geo = tuple(map(int, sys.argv[2].split(","))) if len(sys.argv) > 2 else (0, 2, 64)
    W, H = 1920, 1088
    nmb = (W // 16) * (H // 16)
    clip = synth.clip(W, H, n + 2, 11)
    dev = torch.from_numpy(clip).cuda()
    torch.cuda.synchronize()
    ny, nc = W * H, W * H // 4
    ptrs = [(dev[i].data_ptr(), dev[i].data_ptr() + ny, dev[i].data_ptr() + ny + nc) for i in range(n + 2)]
    enc = Encoder(W, H, 28, 16, 1, 30)
    enc.set_pipeline(*geo)
    if os.environ.get("HL_PROF_HELPERS") == "0":
        enc.set_intra_helpers(False)
    enc.set_timing(True)
    for i in range(2):
        enc.encode_device(*ptrs[i], collect=False)
    enc.profile_counters(64)  # reset
    t = time.perf_counter()
    enc.encode_batch_device(ptrs[2:], collect=False)
    dt = time.perf_counter() - t
    ms = enc.timing_ms()
    nmb_ = nmb
    nsites = int(os.environ.get("HL_BAR_SITES", "0"))  # an HL_BAR_PROF=2 build: 2560 barrier sites after the timeline
    cnt = enc.profile_counters(64 + 4 * nmb_ + 2 * nsites) if nsites else enc.profile_counters(64)
    print(f"wg,R,window={geo}: {n} P pictures in {dt * 1e3:.1f} ms (kernel {ms[1]:.1f} ms, reruns {enc.last_reruns()}) helpers {enc.last_helper_stats()}")
    life, wait, mb, filt, tasks = cnt[44], cnt[40], cnt[41], cnt[42], cnt[43]
    if life:
        wgs = geo[0] or 256
        print(f"   workgroups {wgs}, tasks {tasks} ({tasks / max(1, n * nmb):.2f} per MB), mean lifetime {life / wgs / 1e6:.1f} Mcycles"
              f" (~{life / wgs / (ms[1] * 1e-3) / 1e9:.2f} GHz shader clock if the kernel spans it)")
        hlp, hn = cnt[45], cnt[46]
        print(f"   pops: {cnt[47]} attempts on a macroblock ({cnt[47] / max(1, tasks):.2f} per task), {cnt[48]} lost to another "
              f"workgroup, {cnt[49]} empty rounds ({cnt[49] / max(1, tasks):.1f} per task)")
        if hn:
            print(f"   helper tasks {hn} ({hn / max(1, n * nmb):.2f} per MB), {hlp / hn / 1e3:.1f} kcycles each")
        if cnt[59]:
            print(f"   of which 8x8-family partitioning helpers {cnt[59]}, {cnt[58] / cnt[59] / 1e3:.1f} kcycles each; "
                  f"partitionings the MB found unclaimed {cnt[60]}, still running {cnt[61]} (waited {cnt[63] / max(1, n * nmb) / 1e3:.1f} "
                  f"kcycles/MB), done {cnt[62]}")
        print(f"   after the filters: barrier {cnt[50] / max(1, tasks) / 1e3:.1f}, release fence {cnt[51] / max(1, tasks) / 1e3:.1f}, "
              f"successors {cnt[52] / max(1, tasks) / 1e3:.1f} kcycles/task; early release block (in the filters) {cnt[53] / max(1, tasks) / 1e3:.1f} "
              f"(fence {cnt[54] / max(1, tasks) / 1e3:.1f}, release {cnt[55] / max(1, tasks) / 1e3:.1f}, spin {cnt[56] / max(1, tasks) / 1e3:.1f}, "
              f"acquire {cnt[57] / max(1, tasks) / 1e3:.1f})")
        for name, v in (("task-start waits", wait), ("decisions", mb), ("deblock + planes", filt), ("intra helpers", hlp),
                        ("rest", life - wait - mb - filt - hlp)):
            print(f"   {name:18s} {100.0 * v / life:6.1f} %   {v / max(1, tasks) / 1e3:9.1f} kcycles/task")
    for i, name in enumerate(PHASES):
        cyc, calls = cnt[2 * i], cnt[2 * i + 1]
        if calls and name:
            print(f"   {name:18s} calls/MB {calls / (n * nmb):8.1f}  cycles/call {cyc / calls:10.0f}  kcycles/MB {cyc / (n * nmb) / 1e3:9.1f}")
    if nsites:  # barrier sites by their wait (source line = 2 * site or 2 * site + 1, any header)
        base = 64 + 4 * nmb
        sites = [(cnt[base + 2 * k], cnt[base + 2 * k + 1], k) for k in range(nsites) if cnt[base + 2 * k + 1]]
        tot = sum(w for w, _, _ in sites)
        print(f"   barrier sites: {len(sites)}, wait summed over the waves {tot / (n * nmb) / 1e3:.1f} kcycles/MB")
        for w, c_, k in sorted(sites, reverse=True)[:30]:
            print(f"     line {2 * k:5d}-{2 * k + 1:<5d} calls/MB {c_ / (n * nmb):7.2f}  wait/call (all waves) {w / c_:8.0f}  "
                  f"kcycles/MB {w / (n * nmb) / 1e3:8.1f}  ({100.0 * w / max(1, tot):4.1f} %)")
    enc.close()


if __name__ == "__main__":
    main()
