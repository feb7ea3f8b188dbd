#!/bin/bash
# A/B of the pipelined pop order (HL_AMD_PIPE_HOP: -1 oldest picture first,
# else longest remaining path first with that picture lag) on bench.py's
# workload: bash tools/gpu_hop.sh -1 12 ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for h in "$@"; do
    HL_AMD_PIPE_HOP=$h timeout -k 10 300 python -u tools/ab_bench.py > "gpurun_out/hop_$h.log" 2>&1
    rc=$?
    echo "hop $h: $(grep -v amdgpu.ids "gpurun_out/hop_$h.log" | tail -2 | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
done
