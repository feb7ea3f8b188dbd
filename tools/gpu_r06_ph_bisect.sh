#!/bin/bash
# Round 6: bisecting a bit-exactness failure of the partitioning helpers in
# runs (HL_AMD_FAM3=2 and 3): the family's helpers claimed at its start
# (in-tree) against per partitioning (build/percj).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in hartallo_amd/libhartallo_amd.so build/percj/libhartallo_amd.so; do
  for f3 in 3 2; do
    echo "== $lib HL_AMD_FAM3=$f3"
    HL_LIB=$lib HL_AMD_FAM3=$f3 timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py -k "few_workgroups or equals_single" > gpurun_out/r06_bisect.log 2>&1
    rc=$?; grep -E "passed|failed" gpurun_out/r06_bisect.log | tail -1; [ $rc -le 1 ] || exit $rc
  done
done
