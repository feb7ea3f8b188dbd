"""BASELINE config 5 -- 8 concurrent 1088p IPPP streams, one per GPU -- run
through bench.py's multi-rank path (torch.distributed.run), on the one GPU
of the test box (ranks beyond the visible GPUs share them, bench.py).  Every
stream has its own seed (11-18) and every frame is checked against the
reference encoder's per-frame MD5s for that seed
(tests/golden/bench_golden.json); the line reports the minimum over ranks,
and the summed run statistics show that no rank fell back to the
per-picture path."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_gpus_two_spawns_ranks(gpu):
    """`python bench.py --gpus 2` without torchrun (the driver's command
    form): the launcher starts two ranks (here both on the box's one GPU,
    each with half of its CUs), every frame of both streams (seeds 11, 12)
    bit-exact, and the line names the process group and each rank's device."""
    env = dict(os.environ, OMP_NUM_THREADS="2", HL_AMD_WRITER_THREADS="4")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE"):
        env.pop(k, None)
    cmd = [sys.executable, "bench.py", "--gpus", "2", "--steps", "4", "--warmup", "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 prints the only line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "streams2", line
    assert line["process_group_world_size"] == 2
    assert sorted(x["rank"] for x in line["ranks"]) == [0, 1]
    assert line["distinct_gpus"] == 1  # one GPU on the test box, shared
    assert line["bitexact"] is True, line
    p = line["pipeline"]
    assert p["runs"] == 2 and p["fallbacks"] == 0 and p["waits_gave_up"] == 0, p


def test_config5_eight_streams_share_one_gpu(gpu):
    """The 8 streams (seeds 11-18) at the driver's shape (--warmup 5 --steps
    20 per stream): 2 ranks (processes) of 4 streams each, every rank's
    streams in shared pipelined runs (bench.py --streams 4)."""
    ranks, per_rank, warmup, steps = 2, 4, 5, 20
    env = dict(os.environ, OMP_NUM_THREADS="2", HL_AMD_WRITER_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", str(ranks), "--steps", str(steps), "--warmup", str(warmup),
           "--streams", str(per_rank), "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == ranks and line["config"]["parallelism"] == f"streams{ranks * per_rank}"
    assert line["config"]["streams_per_process"] == per_rank
    assert line["bitexact"] is True, line
    p = line["pipeline"]
    assert p["runs"] == ranks and p["per_picture"] == 0 and p["fallbacks"] == 0 and p["waits_gave_up"] == 0, p
    assert p["warmup_off_pipeline"] == 0, p
