"""BASELINE config 5 -- 8 concurrent 1088p IPPP streams, one per GPU -- run
as the driver runs it, through bench.py's multi-rank path
(torch.distributed.run, one process per stream), with the 8 ranks sharing
the one GPU of the test box (ranks beyond the visible GPUs share them,
bench.py).  Every rank encodes its own seed (11-18) and checks every frame
against the reference encoder's per-frame MD5s for that seed
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
    ranks, warmup, steps = 8, 2, 6
    env = dict(os.environ, OMP_NUM_THREADS="2", HL_AMD_WRITER_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), "bench.py", "--gpus", str(ranks), "--steps", str(steps), "--warmup", str(warmup),
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == ranks and line["config"]["parallelism"] == f"streams{ranks}"
    assert line["bitexact"] is True, line
    p = line["pipeline"]
    assert p["runs"] == ranks and p["per_picture"] == 0 and p["fallbacks"] == 0 and p["waits_gave_up"] == 0, p
    assert p["warmup_off_pipeline"] == 0, p
