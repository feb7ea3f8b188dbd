#!/bin/bash
# Round 6: the 8x8 family's partitionings as four helper tasks (lone
# pictures) against HEAD's single family helper (build/r06base): GPU parity
# (golden streams per call, pipelined runs, the bench stream's MD5s, the
# drop-in), then timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
    tests/test_gpu_bench_golden.py tests/test_drop_in.py > gpurun_out/r06_ph_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_ph_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_bench.py build/r06base/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_ph_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_ph_ab.log; exit $rc
