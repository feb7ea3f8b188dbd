set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 5 60 rocprofv3 -L > gpurun_out/r05b_counters.txt 2>&1; echo "list rc=$?"
timeout -k 10 400 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so build/t256/libhartallo_amd.so > gpurun_out/r05b_ab_t256.log 2>&1 || { tail -5 gpurun_out/r05b_ab_t256.log; exit 1; }
cat gpurun_out/r05b_ab_t256.log | grep -v amdgpu.ids
PMC_SETS="ic:SQC_ICACHE_HITS,SQC_ICACHE_MISSES sq:SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_LDS lds:SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INST_LEVEL_LDS,SQ_IFETCH,SQ_IFETCH_LEVEL,SQ_INSTS_SMEM,SQ_INST_LEVEL_VMEM,SQ_INSTS_VMEM_RD" timeout -k 10 700 bash tools/pmc_ab.sh t256 hartallo_amd/libhartallo_amd.so build/t256/libhartallo_amd.so
python3 tools/pmc_ab_summary.py gpurun_out/pmcab_t256
