#!/bin/bash
# HBM traffic of k_pipeline for library variants (run on the GPU box):
#   bash tools/pmc_traffic_ab.sh lib1.so [lib2.so ...]
# FETCH_SIZE and WRITE_SIZE passes (one counter block each) over
# tools/pipe_bench.py 20 (two warm-up pictures one call at a time, then 20 P
# pictures in one launch); tools/pmc_summary.py --last gives the bytes of the
# 20-picture launch.  Development tool (the write-traffic explanation in
# DESIGN.md).
set -o pipefail
mkdir -p gpurun_out/pmcab
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  for c in FETCH_SIZE WRITE_SIZE; do
    HL_LIB=$R/$lib timeout -s KILL 200 rocprofv3 --pmc $c -d $R/gpurun_out/pmcab/${tag}_$c -o run --output-format csv -- \
        python3 $R/tools/pipe_bench.py 20 > $R/gpurun_out/pmcab/${tag}_$c.log 2>&1 || exit $?
  done
  echo "== $lib"
  grep -h "P pictures" $R/gpurun_out/pmcab/${tag}_WRITE_SIZE.log
  (cd $R && python3 tools/pmc_summary.py --warmup 2 --steps 20 gpurun_out/pmcab/${tag}_FETCH_SIZE gpurun_out/pmcab/${tag}_WRITE_SIZE | grep -E "per_mb")
done
