#!/bin/bash
# Round 6: partitioning helpers for a run's first / last pictures only
# (HL_AMD_FAM3=2, HL_AMD_F3_EDGE=first,last): pipelined-run parity, then the
# driver configuration and 120 frames for several edges against the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HL_AMD_FAM3=2 timeout -k 10 400 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/r06_edge_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_edge_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_edge_default.log 2>&1 || exit $?
for e in 0,0 1,2 1,4 2,6 99,99; do
  HL_AMD_FAM3=2 HL_AMD_F3_EDGE=$e timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_edge_$e.log 2>&1 || exit $?
done
for f in gpurun_out/r06_edge_default.log gpurun_out/r06_edge_[0-9]*.log; do echo "== $f"; grep -v amdgpu.ids $f | grep -v per-picture | cut -c1-150; done
