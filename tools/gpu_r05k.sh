set -o pipefail
bash tools/gpu_ab.sh r05k hartallo_amd/libhartallo_amd.so build/head/libhartallo_amd.so build/subq8/libhartallo_amd.so build/subq16/libhartallo_amd.so build/ldswin/libhartallo_amd.so build/ldsdma/libhartallo_amd.so hartallo_amd/libhartallo_amd.so || exit 1
PMC_SETS="fe:FETCH_SIZE wr:WRITE_SIZE" bash tools/pmc_ab.sh r05k hartallo_amd/libhartallo_amd.so build/ldswin/libhartallo_amd.so build/ldsdma/libhartallo_amd.so || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/pmc_ab_summary.py gpurun_out/pmcab_r05k
