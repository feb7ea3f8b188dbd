#!/bin/bash
# Round 6: the partitioning helpers in runs of one stream (HL_AMD_FAM3=2), the
# in-tree build (helpers only when no macroblock is ready) and one whose
# idle workgroups also take a helper after losing a macroblock race
# (build/ftruns), against the default (lone pictures only).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_phr2_default.log 2>&1 || exit $?
HL_AMD_FAM3=2 timeout -k 10 400 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so build/ftruns/libhartallo_amd.so > gpurun_out/r06_phr2_fam3_2.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_phr2_*.log | grep -v per-picture
