#!/bin/bash
# Round 6: eight column bands for runs of one stream (P.subq 8, in-tree)
# against four (HL_AMD_SUBQ=4): pipelined-run parity, one stream
# (tools/ab_bench.py) and 8 streams in one process.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_streams.py tests/test_gpu_bench_golden.py > gpurun_out/r06_subq_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_subq_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for q in 8 4; do
    HL_AMD_SUBQ=$q timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_subq_$q.log 2>&1 || exit 1
    echo "subq $q: $(grep -v amdgpu.ids gpurun_out/r06_subq_$q.log | grep -v per-picture | cut -c40-75 | tr '\n' ' ')"
    HL_AMD_SUBQ=$q timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 8 > gpurun_out/r06_st8.log 2>&1 || exit 1
    echo "subq $q 8 streams: $(grep '^{' gpurun_out/r06_st8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["bitexact"])')"
  done
done
