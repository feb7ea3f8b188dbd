#!/bin/bash
# Instruction-fetch counters of k_pipeline on the driver workload (bench.py
# --steps 20 --warmup 5), two passes in runs of their own.  Development tool:
#   bash tools/pmc_icache.sh      (GPU box, repo root)
set -o pipefail
mkdir -p gpurun_out/pmci
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
sets=("SQC_ICACHE_HITS SQC_ICACHE_MISSES"
      "SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d $R/gpurun_out/pmci/p$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/pmci/p$i.log 2>&1 || exit $?
done
