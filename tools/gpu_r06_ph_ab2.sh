#!/bin/bash
# Round 6: lone-picture profile with the 8x8 family's partitioning helpers,
# then the A/B against HEAD's build (bit-exact checks included).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=${1:-ph2}
timeout -k 10 200 python3 -u tools/pipe_profile.py 1 > gpurun_out/r06_${tag}_prof.log 2>&1 || { tail -5 gpurun_out/r06_${tag}_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_${tag}_prof.log | head -12
timeout -k 10 600 python3 -u tools/ab_bench.py build/r06base/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_${tag}_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_${tag}_ab.log; exit $rc
