#!/bin/bash
# Round 6: partitioning helpers waited for at each partitioning's start (no
# polling inside the search): A/B against HEAD's build, and the HL_FAM3=1
# kernel in runs without helpers (HL_AMD_FAM3=3).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-phw}
timeout -k 10 600 python3 -u tools/ab_bench.py build/r06base/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_${tag}_ab.log 2>&1 || exit $?
HL_AMD_FAM3=3 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_${tag}_f3k.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_${tag}_ab.log gpurun_out/r06_${tag}_f3k.log
