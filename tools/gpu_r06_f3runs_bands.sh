#!/bin/bash
# Round 6: the partitioning helpers in runs (HL_AMD_FAM3=2; every picture, or
# a run's first and last pictures) on the column-band tree, against the default.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_fb_def.log 2>&1 || exit 1
  echo "default: $(grep -v amdgpu.ids gpurun_out/r06_fb_def.log | grep -v per-picture | cut -c40-75 | tr '\n' ' ')"
  for e in 99,99 1,2; do
    HL_AMD_FAM3=2 HL_AMD_F3_EDGE=$e timeout -k 10 300 python3 -u tools/ab_bench.py hartallo_amd/libhartallo_amd.so > gpurun_out/r06_fb_$e.log 2>&1 || exit 1
    echo "fam3=2 edge $e: $(grep -v amdgpu.ids gpurun_out/r06_fb_$e.log | grep -v per-picture | cut -c40-75 | tr '\n' ' ') $(grep -c 'bitexact True' gpurun_out/r06_fb_$e.log)"
  done
done
