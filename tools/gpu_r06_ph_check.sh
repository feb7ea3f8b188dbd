#!/bin/bash
# Round 6: partitioning helpers + helper sub-FIFOs: GPU parity (golden streams
# per call, pipelined runs, streams, the bench stream's MD5s, the drop-in),
# then the helpers on every run of one stream (HL_AMD_FAM3=2) against the
# default (lone pictures only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
    tests/test_gpu_bench_golden.py tests/test_drop_in.py tests/test_gpu_streams.py > gpurun_out/r06_ph_check_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_ph_check_tests.log; [ $rc -eq 0 ] || exit $rc
HL_AMD_FAM3=2 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_ph_fam3runs.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_ph_fam3runs.log; exit $rc
