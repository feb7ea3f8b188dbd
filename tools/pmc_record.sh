#!/bin/bash
# rocprofv3 PMC counters of k_pipeline on bench.py's driver workload
# (--steps 20 --warmup 5), run on the GPU box from the repo root:
#   bash tools/pmc_record.sh
# Eight passes, each in a run of its own (MI355X_MICROARCH.md: counter slots
# per block, FETCH_SIZE and WRITE_SIZE cannot share a pass): two SQ sets,
# FETCH_SIZE, WRITE_SIZE, and the L2's memory-side request counts by size
# and destination (the read / write byte split, round 6).  tools/pmc_summary.py then writes
# gpurun_out/pmc/pmc_k_pipeline.json (copied to tools/pmc/ by the caller:
# only gpurun_out/ comes back from the GPU box) for the timed launch (the
# last k_pipeline dispatch), stamped with the SHA-256 of the library it
# measured; bench.py uses the counters only when that hash is the loaded
# library's.
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
sets=("SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
      "SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM"
      "FETCH_SIZE" "WRITE_SIZE"
      "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
      "TCC_EA0_WRREQ_WRITE_IO_32B_sum TCC_EA0_WRREQ_ATOMIC_DRAM_sum" "TCC_EA0_WRREQ_WRITE_DRAM_sum")
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set -d $R/gpurun_out/pmc/p$i -o run --output-format csv -- \
      python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/pmc/p$i.log 2>&1 || exit $?
done
cd $R
python3 tools/pmc_summary.py --warmup 5 --steps 20 --width 1920 --height 1088 --workgroups 0 --streams-per-gpu 1 gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/p3 gpurun_out/pmc/p4 \
    gpurun_out/pmc/p5 gpurun_out/pmc/p6 gpurun_out/pmc/p7 gpurun_out/pmc/p8 \
    > gpurun_out/pmc/pmc_k_pipeline.json && cat gpurun_out/pmc/pmc_k_pipeline.json
