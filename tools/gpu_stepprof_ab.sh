# step-profile (HL_PROFILE + HL_STEP_PROF builds) of several libraries on
# the driver's 20-picture run: bash tools/gpu_stepprof_ab.sh tag lib...
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for lib in "$@"; do
  i=$((i+1))
  HL_LIB=$lib HL_STEP_NAMES=1 timeout -k 10 200 python3 -u tools/pipe_profile.py 20 > gpurun_out/${tag}_$i.log 2>&1 || { tail -3 gpurun_out/${tag}_$i.log; exit 1; }
  echo "== $lib"; grep -v amdgpu.ids gpurun_out/${tag}_$i.log | grep "whole MB\|step:\|eval:\|search_partition\|guess_intra\|P pictures in"
done
