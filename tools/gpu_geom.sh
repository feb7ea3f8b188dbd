#!/bin/bash
# A/B of pipelined-run geometries (hl_amd_set_pipeline: workgroups,reach,window)
# on bench.py's workload: bash tools/gpu_geom.sh "0,2,64" "0,1,64" ...
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for g in "$@"; do
    HL_AB_GEOM=$g timeout -k 10 300 python -u tools/ab_bench.py > "gpurun_out/geom_$g.log" 2>&1
    rc=$?
    grep -v amdgpu.ids "gpurun_out/geom_$g.log" | tail -3
    [ $rc -eq 0 ] || exit $rc
done
