#!/bin/bash
# Quick GPU check after a kernel change: parity suites (per-picture, pipelined,
# reference MD5s at the BASELINE sizes), the A/B bench (tools/ab_bench.py) and
# a rocprofv3 kernel summary of a short bench.  Outputs under gpurun_out/q_*.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/q_$name.log" 2>&1
    local rc=$?
    grep -v amdgpu.ids "gpurun_out/q_$name.log" | tail -${TAILN:-4}
    echo "== $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_bench_golden.py
TAILN=6 step ab 600 python -u tools/ab_bench.py "$@"
step prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/q_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
