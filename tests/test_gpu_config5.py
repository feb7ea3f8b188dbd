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
