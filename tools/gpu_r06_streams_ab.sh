#!/bin/bash
# Round 6: 8 streams in one process (bench.py --streams 8, the driver's shape)
# with the in-tree build and build/r06ph4 (address-interleaved sub-queues), twice each
# (the box's copy of the tree gets each library in turn).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp hartallo_amd/libhartallo_amd.so /tmp/base_lib.so
for rep in 1 2; do
  for lib in /tmp/base_lib.so build/r06ph4/libhartallo_amd.so; do
    cp $lib hartallo_amd/libhartallo_amd.so
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 8 > gpurun_out/r06_st8.log 2>&1 || { tail -3 gpurun_out/r06_st8.log; exit 1; }
    echo "$lib $(grep '^{' gpurun_out/r06_st8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["bitexact"])')"
  done
done
cp /tmp/base_lib.so hartallo_amd/libhartallo_amd.so
