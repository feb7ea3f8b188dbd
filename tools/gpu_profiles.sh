# tools/pipe_profile.py on several profiling builds (20-picture driver run):
#   bash tools/gpu_profiles.sh tag lib.so:ENV=1 [lib.so:ENV=1 ...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  i=$((i+1)); lib=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=
  env HL_LIB=$lib $envs timeout -k 10 200 python3 -u tools/pipe_profile.py 20 > gpurun_out/${tag}_$i.log 2>&1 || { tail -3 gpurun_out/${tag}_$i.log; exit 1; }
  echo "== $spec"; grep -v amdgpu.ids gpurun_out/${tag}_$i.log
done
