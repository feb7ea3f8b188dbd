#!/bin/bash
# Round 6: the partitioning helpers as kept (waited for at each partitioning's
# start, claimed per partitioning): GPU parity (default, and the pipelined-run
# tests with the helpers in runs, HL_AMD_FAM3=2), the A/B against HEAD~ and
# the helpers in runs.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
    tests/test_gpu_bench_golden.py tests/test_drop_in.py tests/test_gpu_streams.py > gpurun_out/r06_phf_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_phf_tests.log; [ $rc -eq 0 ] || exit $rc
HL_AMD_FAM3=2 timeout -k 10 400 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/r06_phf_tests_fam3runs.log 2>&1
rc=$?; tail -2 gpurun_out/r06_phf_tests_fam3runs.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_bench.py build/r06base/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phf_ab.log 2>&1 || exit $?
HL_AMD_FAM3=2 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phf_fam3runs.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_phf_ab.log gpurun_out/r06_phf_fam3runs.log | cut -c1-260
