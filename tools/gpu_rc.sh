#!/bin/bash
# GPU check after the rate-control change: parity suites (golden streams incl.
# rate control, drop-in through hl_codec_encode, pipelined runs, reference
# MD5s at the BASELINE sizes) and the A/B bench.  Outputs gpurun_out/rc_*.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/rc_$name.log" 2>&1
    local rc=$?
    grep -v amdgpu.ids "gpurun_out/rc_$name.log" | tail -${TAILN:-4}
    echo "== $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
step tests 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_drop_in.py tests/test_gpu_pipeline.py tests/test_gpu_bench_golden.py
TAILN=6 step ab 600 python -u tools/ab_bench.py
