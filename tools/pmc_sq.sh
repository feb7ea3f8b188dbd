# SQ latency/stall counters of the pipelined kernel (development tool; run via gpurun)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $GRAFT_REPO_ROOT/gpurun_out/sq$i -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/pipe_bench.py 12 > $GRAFT_REPO_ROOT/gpurun_out/sq$i.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, collections
for i in (1, 2):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(f"gpurun_out/sq{i}/run_counter_collection.csv")):
        if r["Kernel_Name"].startswith("k_pipeline"):
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in sorted(acc.items()):
        print(f"{k:24s} {v:.4g}")
PY
