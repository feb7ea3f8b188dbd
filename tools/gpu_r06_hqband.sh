#!/bin/bash
# Round 6: a lone picture's helper FIFOs by column band (in-tree) against the
# even spread (HL_AMD_HQ_SPREAD=1): parity (per-call goldens, drop-in), then
# tools/ab_bench.py (its per-picture line) twice each.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_golden.py tests/test_drop_in.py > gpurun_out/r06_hqb_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_hqb_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_hqb_band.log 2>&1 || exit 1
  echo "band:   $(grep -v amdgpu.ids gpurun_out/r06_hqb_band.log | cut -c40-100 | tr '\n' '|')"
  HL_AMD_HQ_SPREAD=1 timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_hqb_spread.log 2>&1 || exit 1
  echo "spread: $(grep -v amdgpu.ids gpurun_out/r06_hqb_spread.log | cut -c40-100 | tr '\n' '|')"
done
