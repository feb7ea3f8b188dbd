# gpu_ab.sh, then one tools/pipe_profile.py run of a profiling build:
#   PROF_LIB=build/x/lib.so PROF_ENV="HL_I4_NAMES=1" bash tools/gpu_ab_prof.sh tag lib1.so [lib2.so ...]
set -o pipefail
tag=$1
bash "$(dirname "$0")/gpu_ab.sh" "$@" || exit 1
cd "$GRAFT_REPO_ROOT"
env HL_LIB=$PROF_LIB $PROF_ENV timeout -k 10 200 python3 -u tools/pipe_profile.py 20 > gpurun_out/${tag}_prof.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${tag}_prof.log; exit $rc
