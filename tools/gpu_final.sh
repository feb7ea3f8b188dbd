#!/bin/bash
# End-of-session GPU pass (GPU box, repo root): bash tools/gpu_final.sh <tag>
# -m gpu suite, smoke, driver-config and default benches, rocprofv3 kernel
# summary (tools/gpu_round.sh), the per-frame path through the reference's
# API, the SVC bench (config 4, one GPU), PMC counters of the shipped library
# (tools/pmc_record.sh, recorded first) and one vs two streams sharing the GPU.
set -o pipefail
tag=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# counters first, copied into this box's tools/pmc/ so that the bench lines
# below already carry them (the copy under gpurun_out/ comes back)
echo "== pmc"
bash tools/pmc_record.sh > gpurun_out/${tag}_pmc_record.log 2>&1 || { tail -5 gpurun_out/${tag}_pmc_record.log; exit 1; }
grep "sq_\|valu_insts\|traffic_bytes_per_mb\|lib_sha" gpurun_out/${tag}_pmc_record.log
cp gpurun_out/pmc/pmc_k_pipeline.json tools/pmc/pmc_k_pipeline.json
bash tools/gpu_round.sh $tag || exit 1
echo "== per-frame API"
timeout -k 10 200 python -u tools/per_frame_api.py 8 > gpurun_out/${tag}_per_frame_api.log 2>&1 || { tail -5 gpurun_out/${tag}_per_frame_api.log; exit 1; }
grep '^{' gpurun_out/${tag}_per_frame_api.log
echo "== svc"
timeout -k 10 300 python -u bench.py --svc > gpurun_out/${tag}_svc_bench.log 2>&1 || { tail -5 gpurun_out/${tag}_svc_bench.log; exit 1; }
grep '^{' gpurun_out/${tag}_svc_bench.log | cut -c1-300
echo "== share"
NS="1 2" bash tools/gpu_share.sh
