set -o pipefail
tag=${1:-svcprof}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/svc_profile.py 20 > gpurun_out/${tag}_calls.log 2>&1 || { tail -20 gpurun_out/${tag}_calls.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_calls.log | tail -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof -o run --output-format csv -- python3 bench.py --svc > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
f=$(find gpurun_out/${tag}_prof -name "*kernel_stats.csv" | head -1); head -12 "$f"
