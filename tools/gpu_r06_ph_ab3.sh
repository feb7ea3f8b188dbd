#!/bin/bash
# Round 6: lone-picture profile and A/B of the in-tree build against a base
# build (bit-exact checks included): bash tools/gpu_r06_ph_ab3.sh <tag> <base.so>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=$1; base=$2
timeout -k 10 200 python3 -u tools/pipe_profile.py 1 > gpurun_out/r06_${tag}_prof.log 2>&1 || { tail -5 gpurun_out/r06_${tag}_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_${tag}_prof.log | head -14
timeout -k 10 600 python3 -u tools/ab_bench.py $base hartallo_amd/libhartallo_amd.so > gpurun_out/r06_${tag}_ab.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_${tag}_ab.log | cut -c1-220; exit $rc
