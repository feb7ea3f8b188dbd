#!/bin/bash
# rocprofv3 counter passes of k_pipeline for several library builds on the
# driver workload (tools/run_lib.py: 5 + 20 pictures), one pass per run
# (MI355X_MICROARCH.md: counters per block).  Development tool, GPU box:
#   bash tools/pmc_ab.sh tag lib1.so [lib2.so ...]
# Each set is "NAME:counters"; the summary is tools/pmc_ab_summary.py.
set -o pipefail
tag=$1
shift
mkdir -p gpurun_out/pmcab_$tag
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
sets=(${PMC_SETS:-"ic:SQC_ICACHE_HITS,SQC_ICACHE_MISSES" "sq:SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAIT_INST_LDS"})
li=0
for lib in "$@"; do
  li=$((li+1))
  for s in "${sets[@]}"; do
    name=${s%%:*}
    ctr=${s#*:}
    d=$R/gpurun_out/pmcab_$tag/l${li}_$name
    timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d $d -o run --output-format csv -- \
        python3 $R/tools/run_lib.py $R/$lib > $d.log 2>&1 || { echo "pass $lib $name failed"; tail -3 $d.log; exit 1; }
    echo "$lib $name: $(grep '^{' $d.log)"
  done
done
