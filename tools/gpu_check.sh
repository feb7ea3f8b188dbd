# GPU-box check: unit + parity tests, a short bench and (optionally) the phase
# profile of the HL_PROFILE build.  Run via gpurun from the repo root:
#   bash tools/gpu_check.sh [profile]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_unit.py tests/test_gpu_parity.py > gpurun_out/parity.log 2>&1
rc=$?
tail -8 gpurun_out/parity.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/bench.log
if [ "$1" = "profile" ]; then
  timeout -k 10 200 python -u tools/phase_profile.py 3 > gpurun_out/phase.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/phase.log | tail -14
fi
