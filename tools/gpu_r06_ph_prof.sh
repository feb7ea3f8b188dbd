#!/bin/bash
# Round 6: where a lone picture's workgroups spend their time with the 8x8
# family's partitioning helpers (profiling build), and without them.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python3 -u tools/pipe_profile.py 1 > gpurun_out/r06_ph_prof.log 2>&1 || { tail -5 gpurun_out/r06_ph_prof.log; exit 1; }
HL_AMD_FAM3=0 timeout -k 10 200 python3 -u tools/pipe_profile.py 1 > gpurun_out/r06_ph_prof_off.log 2>&1 || { tail -5 gpurun_out/r06_ph_prof_off.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_ph_prof.log; echo "== HL_AMD_FAM3=0"; grep -v amdgpu.ids gpurun_out/r06_ph_prof_off.log
