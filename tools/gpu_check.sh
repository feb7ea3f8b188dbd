# GPU-box check: unit + parity tests, then a short bench (run via gpurun from the repo root)
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_unit.py tests/test_gpu_parity.py > gpurun_out/parity.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?
tail -25 gpurun_out/parity.log; cat gpurun_out/bench.log | tail -3
exit $rc
