#!/bin/bash
# Round 6: the partitioning helpers' entry guess of one coefficient per block
# (hl_mbcore.h encode_mb): GPU suite, per-call probe and per-frame API, the
# default benches (ab_bench.py), and the helpers in runs (HL_AMD_FAM3=2,
# every picture) against them.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests > gpurun_out/r06g1_tests.log 2>&1 || { tail -20 gpurun_out/r06g1_tests.log; exit 1; }
tail -1 gpurun_out/r06g1_tests.log
timeout -k 10 200 python3 -u tools/per_call_probe.py 10 > gpurun_out/r06g1_probe.log 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/per_frame_api.py 8 > gpurun_out/r06g1_per_frame_api.log 2>&1 || exit $?
grep '^{' gpurun_out/r06g1_per_frame_api.log | cut -c1-330
timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06g1_default.log 2>&1 || exit $?
HL_AMD_FAM3=2 HL_AMD_F3_EDGE=99,99 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06g1_runs_fam3.log 2>&1 || exit $?
for f in gpurun_out/r06g1_default.log gpurun_out/r06g1_runs_fam3.log; do echo "== $f"; grep -v amdgpu.ids $f | cut -c1-190; done
