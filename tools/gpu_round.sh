#!/bin/bash
# Full GPU check, run on the GPU box from the repo root:
#   bash tools/gpu_round.sh <tag>
# the -m gpu suite, smoke(), the default bench and the driver's bench
# configuration, and a rocprofv3 kernel-trace summary of the default bench.
# Outputs under gpurun_out/<tag>_*; every GPU step has its own time limit and
# the script stops at the first failure.
set -o pipefail
tag=${1:-run}
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
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench_driver 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
step bench 400 python -u bench.py
step prof 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/${tag}_prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline
