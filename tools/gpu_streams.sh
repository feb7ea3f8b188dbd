#!/bin/bash
# Several streams per GPU in one process (hl_amd_encode_streams), on the GPU
# box from the repo root: the stream tests, then bench.py's driver shape with
# 1, 2 and 4 streams per process (and 8: config 5 on one GPU).  Outputs under
# gpurun_out/s_*.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/s_$name.log" 2>&1
    local rc=$?
    grep -v amdgpu.ids "gpurun_out/s_$name.log" | tail -${TAILN:-3} | cut -c1-600
    echo "== $name rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_streams.py tests/test_gpu_config5.py
for k in ${STREAMS:-1 2 4 8}; do
    step bench_k$k 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams $k
done
