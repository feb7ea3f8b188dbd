#!/bin/bash
# Round 6: the partitioning helpers in runs (HL_AMD_FAM3=2): pipelined-run
# parity (tests/test_gpu_pipeline.py) of the in-tree build and of HEAD's
# (build/r06ph: helpers polled inside the search), then bench-stream MD5s.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for lib in build/r06ph/libhartallo_amd.so hartallo_amd/libhartallo_amd.so; do
  echo "== $lib"
  HL_LIB=$lib HL_AMD_FAM3=2 timeout -k 10 400 python3 -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/r06_race_$(basename $(dirname $lib)).log 2>&1
  rc=$?; tail -4 gpurun_out/r06_race_$(basename $(dirname $lib)).log; [ $rc -le 1 ] || exit $rc
done
HL_AMD_FAM3=2 timeout -k 10 400 python3 -u tools/ab_bench.py build/r06ph/libhartallo_amd.so hartallo_amd/libhartallo_amd.so build/r06ph/libhartallo_amd.so hartallo_amd/libhartallo_amd.so > gpurun_out/r06_race_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r06_race_ab.log | grep -v per-picture | cut -c1-200
