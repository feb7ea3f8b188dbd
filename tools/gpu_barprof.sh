# barrier-wait profile (HL_BAR_PROF build) of the driver's 20-picture run, and
# VALU lane utilisation / L1-L2 read latency counters of the product
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HL_LIB=build/barprof/libhartallo_amd.so HL_BAR_NAMES=1 timeout -k 10 300 python3 -u tools/pipe_profile.py 20 > gpurun_out/r05c_barprof.log 2>&1 || { tail -5 gpurun_out/r05c_barprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r05c_barprof.log
PMC_SETS="va:SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_VMEM,SQ_INST_CYCLES_SALU,SQ_ACTIVE_INST_MISC,SQ_BUSY_CYCLES tcp:TCP_TCC_READ_REQ_LATENCY_sum,TCP_TCC_READ_REQ_sum,TCP_TOTAL_CACHE_ACCESSES_sum,TCP_CACHE_MISS_sum" timeout -k 10 400 bash tools/pmc_ab.sh va hartallo_amd/libhartallo_amd.so build/t256/libhartallo_amd.so
python3 tools/pmc_ab_summary.py gpurun_out/pmcab_va
