#!/bin/bash
# Round 6 diagnostic: the HL_FAM3=1 kernel in runs without helpers
# (HL_AMD_FAM3=3): in-tree build against one with the helper path compiled out.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HL_AMD_FAM3=3 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so build/f3nohelp/libhartallo_amd.so > gpurun_out/r06_f3diag.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_f3diag.log | grep -v per-picture; exit $rc
