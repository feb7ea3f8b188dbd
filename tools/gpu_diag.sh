#!/bin/bash
# A/B of library variants on the GPU box (tools/ab_bench.py) after a parity
# pass of the variant (pipeline goldens + bench goldens).
set -o pipefail
mkdir -p gpurun_out
run() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/diag_$name.log" 2>&1
    local rc=$?
    grep -v amdgpu.ids "gpurun_out/diag_$name.log" | tail -${TAILN:-3}
    echo "== $name rc=$rc"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for v in "$@"; do
    HL_LIB=build/$v/libhartallo_amd.so run parity_$v 400 $T tests/test_gpu_pipeline.py tests/test_gpu_parity.py tests/test_gpu_bench_golden.py -k "golden or driver or 720p"
done
TAILN=20 run ab 900 python -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so $(for v in "$@"; do echo build/$v/libhartallo_amd.so; done)
