# GPU-box check of a kernel change: parity of the pipelined and per-call
# paths, then timing (pipelined run of 28 P pictures, isolated search steps).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_unit.py > gpurun_out/perf_tests.log 2>&1
rc=$?
tail -3 gpurun_out/perf_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/pipe_bench.py 28 > gpurun_out/perf_pb.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/perf_pb.log
if [ -x build/stepbench ]; then timeout -k 5 60 ./build/stepbench > gpurun_out/perf_step.log 2>&1 || exit $?; cat gpurun_out/perf_step.log; fi
