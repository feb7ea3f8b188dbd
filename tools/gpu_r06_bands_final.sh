#!/bin/bash
# Round 6: column bands for one stream only (in-tree) against address-
# interleaved sub-queues (build/r06ph4) and bands for every stream count
# (build/bands4b): 8 streams in one process, then tools/ab_bench.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
cp hartallo_amd/libhartallo_amd.so /tmp/base_lib.so
for lib in /tmp/base_lib.so build/r06ph4/libhartallo_amd.so /tmp/base_lib.so build/r06ph4/libhartallo_amd.so; do
  cp $lib hartallo_amd/libhartallo_amd.so
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 8 > gpurun_out/r06_st8.log 2>&1 || { tail -3 gpurun_out/r06_st8.log; exit 1; }
  echo "8 streams: $lib $(grep '^{' gpurun_out/r06_st8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.readline()); print(d["value"], d["bitexact"])')"
done
cp /tmp/base_lib.so hartallo_amd/libhartallo_amd.so
timeout -k 10 900 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so build/r06ph4/libhartallo_amd.so build/bands4b/libhartallo_amd.so hartallo_amd/libhartallo_amd.so build/r06ph4/libhartallo_amd.so build/bands4b/libhartallo_amd.so > gpurun_out/r06_bands_final.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r06_bands_final.log | grep -v per-picture | cut -c1-100; exit $rc
