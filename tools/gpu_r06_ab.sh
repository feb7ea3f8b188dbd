#!/bin/bash
# Round 6: generic A/B of library builds (tools/ab_bench.py, bit-exact checks
# included): bash tools/gpu_r06_ab.sh <tag> <lib.so> ...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python3 -u tools/ab_bench.py "$@" > gpurun_out/r06_${tag}.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_${tag}.log | cut -c1-200; exit $rc
