# Lists available counters and collects instruction-cache / wait counters
# for a short encode (development tool; run via gpurun from the repo root).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1
cd $GRAFT_REPO_ROOT
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVES SQ_WAVE_CYCLES" "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set -d gpurun_out/pmc_$tag -o run --output-format csv -- python3 tools/quick_bench.py hartallo_amd/libhartallo_amd.so 2 > gpurun_out/pmc_$tag.log 2>&1 || echo "pass $tag failed rc=$?"
done
ls -R gpurun_out | head -50
