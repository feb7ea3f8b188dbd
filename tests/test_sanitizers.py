"""Sanitizer runs of the host code (CPU).

* AddressSanitizer over the emulator (the product's macroblock kernel logic
  run on the host, tests/emu) with the product's host writer (hl_writer.cpp)
  and rate controller (hl_rc.cpp) under AddressSanitizer +
  UndefinedBehaviorSanitizer (tests/sanitize/libhl_emu_asan.so, `make
  sanitize`): the emulator golden suite re-run in a child process with the
  clang ASan runtime preloaded; any report aborts it.  When the 16-minute
  `make ubsan` build (the kernel logic under UBSan too) is present, it is
  used instead.
* ThreadSanitizer over the pipelined run's slice writers
  (tests/sanitize/rowgate_tsan.cpp): row-gated write_slice threads against a
  producer that publishes rows the way k_pipeline does; the gated slices
  must equal the slices written afterwards and TSan must report nothing --
  and a negative control with relaxed publication must be flagged.
"""
import glob
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = os.path.join(HERE, "sanitize")
ASAN_LIB = os.path.join(SAN, "libhl_emu_asan.so")
UBSAN_LIB = os.path.join(SAN, "libhl_emu_ubsan.so")
TSAN_BIN = os.path.join(SAN, "rowgate_tsan")


def _built(path):
    if not os.path.exists(path):  # build() makes them; a bare pytest run builds here (about a minute)
        subprocess.run(["make", "-C", ROOT, "-j4", "sanitize"], check=True, capture_output=True)
    assert os.path.exists(path), f"{path}: `make sanitize` did not build it"
    return path


def _asan_runtime():
    rts = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so")
    if not rts:
        pytest.skip("the clang ASan runtime of the ROCm toolchain is not installed")
    return rts[0]


def test_emulator_goldens_under_asan_ubsan():
    lib = UBSAN_LIB if os.path.exists(UBSAN_LIB) else _built(ASAN_LIB)
    env = dict(os.environ, LD_PRELOAD=_asan_runtime(), HL_EMU_LIB=lib,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    env.pop("PYTEST_ADDOPTS", None)
    # the golden streams (every configuration up to CIF: rate control, early
    # termination, max_ref_frame, SVC, helpers with right and wrong guesses)
    # and the tile deblocking against the raster filter
    code = ("import sys, pytest; sys.exit(pytest.main(['-q', '-s', '-x', '-p', 'no:cacheprovider', "
            "'tests/test_emu_golden.py', 'tests/test_emu_svc.py', 'tests/test_emu_deblock.py', "
            "'-k', 'not 720p and not w480 and not 1088']))")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    report = [ln for ln in (r.stdout + r.stderr).splitlines() if "Sanitizer" in ln or "runtime error" in ln]
    assert r.returncode == 0 and not report, f"status {r.returncode}: {report[:6] or r.stdout[-2000:]}"
    assert " passed" in r.stdout


def test_row_gated_writers_under_tsan():
    exe = _built(TSAN_BIN)
    env = dict(os.environ, TSAN_OPTIONS="history_size=7:halt_on_error=1")
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "rowgate ok" in r.stdout


def test_tsan_flags_relaxed_publication():
    """Negative control: the same run with the row count published and read
    relaxed has no happens-before edge to the records; TSan must see it."""
    exe = _built(TSAN_BIN)
    env = dict(os.environ, TSAN_OPTIONS="history_size=7")
    r = subprocess.run([exe, "relaxed"], env=env, capture_output=True, text=True, timeout=300)
    assert "WARNING: ThreadSanitizer: data race" in r.stderr and "write_slice" in r.stderr
