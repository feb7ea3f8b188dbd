#!/bin/bash
# Round 6: the partitioning helpers in runs of one stream: HL_AMD_FAM3=2 (no
# lost-race fallthrough in runs) and 3 (their kernel build in runs, no helpers
# queued) against the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phr_default.log 2>&1 || exit $?
HL_AMD_FAM3=2 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phr_fam3_2.log 2>&1 || exit $?
HL_AMD_FAM3=3 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phr_fam3_3.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_phr_*.log | grep -v per-picture
