#!/bin/bash
# PMC passes of the pipelined kernel (HBM traffic, SQ issue/wait counters);
# each counter set in its own rocprofv3 run, each bounded by timeout.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_traffic.sh && bash tools/pmc_sq.sh > gpurun_out/pmc_sq_summary.txt && cat gpurun_out/pmc_sq_summary.txt
