#!/bin/bash
# Round 6: Intra4x4 neighbours through ds_bpermute (HL_I4_BPERM=1, the
# in-tree product) against the LDS round trip (build/i4lds): GPU parity
# (golden streams, pipelined runs, the bench stream's MD5s), then timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
    tests/test_gpu_bench_golden.py > gpurun_out/r06_i4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06_i4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_bench.py build/i4lds/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_i4_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_i4_ab.log; exit $rc
