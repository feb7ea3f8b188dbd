# Quick GPU-box check after a change to the pipelined path: its parity
# tests, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py > gpurun_out/quick_tests.log 2>&1
rc=$?
tail -3 gpurun_out/quick_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/bench.log
