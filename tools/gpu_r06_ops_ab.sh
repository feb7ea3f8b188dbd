#!/bin/bash
# Round 6: op-level parity against the reference's own kernels
# (tests/test_gpu_ops.py), then tools/ab_bench.py with the 8x8-family helper
# build on lone pictures only (default) and on every run of one stream
# (HL_AMD_FAM3=2).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py > gpurun_out/r06_ops.log 2>&1
rc=$?; tail -12 gpurun_out/r06_ops.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_ab_base.log 2>&1 || exit $?
HL_AMD_FAM3=2 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_ab_fam3runs.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_ab_*.log
