"""bench.py's rank launcher (CPU): `python bench.py --gpus N` without
torchrun starts N rank processes itself (one per GPU, RANK = LOCAL_RANK =
r, WORLD_SIZE = N) and never touches a GPU in the launching process; under
torchrun an explicit --gpus that disagrees with WORLD_SIZE is refused.  The
GPU side (two ranks sharing the test box's GPU, bit-exact) is
tests/test_gpu_config5.py::test_bench_gpus_two_spawns_ranks."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_resolve_world(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.resolve_world(None) == (1, False)
    assert bench.resolve_world(1) == (1, False)
    assert bench.resolve_world(8) == (8, True)
    with pytest.raises(SystemExit):
        bench.resolve_world(0)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert bench.resolve_world(None) == (4, False)
    assert bench.resolve_world(4) == (4, False)
    with pytest.raises(SystemExit):
        bench.resolve_world(2)


def test_world_size_mismatch_exits_nonzero():
    """torchrun's WORLD_SIZE=2 with --gpus 3: a loud failure before any
    work, not a one-rank run reported as three GPUs."""
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--steps", "1", "--warmup", "0"], cwd=ROOT,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 3" in r.stderr


def test_spawn_ranks_environment(tmp_path):
    """Every rank gets its own RANK / LOCAL_RANK, the shared world size and
    one rendezvous address, and the launcher's status is 0 when all ranks
    succeed."""
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text(
        "import json, os, sys\n"
        "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')\n"
        f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write(json.dumps({{k: os.environ[k] for k in keys}} | {{'argv': sys.argv[1:]}}))\n")
    assert bench.spawn_ranks(3, ["--gpus", "3", "--steps", "2"], script=str(probe)) == 0
    got = [json.loads((out / str(r)).read_text()) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] and [g["LOCAL_RANK"] for g in got] == ["0", "1", "2"]
    assert all(g["WORLD_SIZE"] == "3" and g["LOCAL_WORLD_SIZE"] == "3" and g["MASTER_ADDR"] == "127.0.0.1" for g in got)
    assert len({g["MASTER_PORT"] for g in got}) == 1
    assert all(g["argv"] == ["--gpus", "3", "--steps", "2"] for g in got)


def test_spawn_ranks_failure_stops_the_others(tmp_path):
    """Rank 1 fails; rank 0 would wait forever at a collective: it is
    terminated and the launcher returns rank 1's status."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                     "time.sleep(600)\n")
    assert bench.spawn_ranks(2, [], script=str(probe)) == 3


def test_spawn_ranks_straggler_after_clean_exit(tmp_path, monkeypatch):
    """Rank 1 exits 0 while rank 0 hangs (a peer stuck at a collective or on
    the GPU): after the grace period rank 0 is stopped (SIGTERM, then SIGKILL
    if it ignores it) and the status is non-zero."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, signal, sys, time\n"
                     "if os.environ['RANK'] == '1':\n    sys.exit(0)\n"
                     "signal.signal(signal.SIGTERM, signal.SIG_IGN)\n"
                     "time.sleep(600)\n")
    monkeypatch.setenv("HL_BENCH_GRACE", "1")
    t = time.monotonic()
    assert bench.spawn_ranks(2, [], script=str(probe)) == 124
    assert time.monotonic() - t < 60


def test_spawn_ranks_deadline(tmp_path, monkeypatch):
    """Every rank hangs: the whole-group deadline stops them."""
    probe = tmp_path / "probe.py"
    probe.write_text("import time\ntime.sleep(600)\n")
    monkeypatch.setenv("HL_BENCH_TIMEOUT", "2")
    t = time.monotonic()
    assert bench.spawn_ranks(2, [], script=str(probe)) == 124
    assert time.monotonic() - t < 60


def test_pmc_record_identity(tmp_path, monkeypatch):
    """bench.load_pmc: the counters are used on the library they were taken
    on, or on a relink of the same code (only the ELF string tables differ);
    a library with other code, or another workload, gets none."""
    from hartallo_amd import _lib

    lib = os.path.join(ROOT, "hartallo_amd", "libhartallo_amd.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    code = _lib.code_sha256(lib)
    rec = {"lib_sha256": "0" * 64, "code_sha256": code, "warmup": 1, "steps": 2, "workgroups": 0, "streams_per_gpu": 1,
           "width": bench.W, "height": bench.H, "recorded": "x"}
    f = tmp_path / "pmc.json"
    f.write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "PMC_FILE", str(f))
    pmc, why = bench.load_pmc(lib, 1, 2, 0, 1)
    assert pmc is not None and "code sha256" in why
    assert bench.load_pmc(lib, 1, 3, 0, 1)[0] is None  # another workload
    f.write_text(json.dumps(dict(rec, code_sha256="1" * 64)))
    pmc, why = bench.load_pmc(lib, 1, 2, 0, 1)
    assert pmc is None and why.startswith("stale")
    # a copy with a string-table byte changed keeps the code hash
    data = bytearray(open(lib, "rb").read())
    data[-1] ^= 0xFF  # the section header table ends the file; its last field is sh_entsize of the last section
    other = tmp_path / "relink.so"
    other.write_bytes(bytes(data))
    assert _lib.code_sha256(str(other)) == code
