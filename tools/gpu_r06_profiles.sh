#!/bin/bash
# Round 6 baseline profiles of the pipelined driver run (20 P pictures):
# default profiling build, step sub-phases, Intra4x4 sub-phases, barriers.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # tag lib env...
  local tag=$1 lib=$2; shift 2
  env HL_LIB=$lib "$@" timeout -k 10 200 python3 -u tools/pipe_profile.py 20 > gpurun_out/r06_prof_$tag.log 2>&1 || { tail -3 gpurun_out/r06_prof_$tag.log; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids gpurun_out/r06_prof_$tag.log
}
run default build/prof/hartallo_amd/libhartallo_amd.so
run step build/stepprof/libhartallo_amd.so HL_STEP_NAMES=1
run i4 build/i4prof/libhartallo_amd.so HL_I4_NAMES=1
run bar build/barprof/libhartallo_amd.so HL_BAR_NAMES=1
