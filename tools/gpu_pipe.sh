# GPU-box check of the pipelined path: pipeline parity tests, then a quick timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipeline.py > gpurun_out/pipe.log 2>&1
rc=$?
tail -25 gpurun_out/pipe.log
exit $rc
