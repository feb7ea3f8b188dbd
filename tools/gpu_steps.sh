#!/bin/bash
# Runs named GPU steps on the GPU box from the repo root, each under its own
# time limit, stopping at the first failure:
#   bash tools/gpu_steps.sh <tag> <step> [<step> ...]
# steps: tests smoke bench_driver bench per_frame per_frame720 prof pmc svc
# Outputs under gpurun_out/<tag>_<step>.log (+ gpurun_out/<tag>_prof/).
set -o pipefail
tag=${1:-run}
shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
    local rc=$?
    grep -v amdgpu.ids "gpurun_out/${tag}_$name.log" | tail -4
    echo "== $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
for s in "$@"; do
    case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_driver) step bench_driver 400 python -u bench.py --steps 20 --warmup 5 ;;
    bench) step bench 400 python -u bench.py --no-cpu-baseline ;;
    per_frame) step per_frame 300 python -u tools/per_frame_api.py 8 bench_1088p_s11 ;;
    per_frame720) step per_frame720 300 python -u tools/per_frame_api.py 8 c2_720p_s7 ;;
    svc) step svc 400 python -u bench.py --svc --no-cpu-baseline ;;
    prof) step prof 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    pmc) step pmc 900 bash tools/pmc_record.sh ;;
    phase) step phase 400 python -u tools/phase_profile.py ;;
    pipe) step pipe 400 python -u tools/pipe_profile.py ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
