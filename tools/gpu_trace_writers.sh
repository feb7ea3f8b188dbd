set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HL_AMD_TRACE_WRITERS=1 timeout -k 10 300 python -u tools/ab_bench.py > gpurun_out/trace_writers.log 2>&1
rc=$?; tail -5 gpurun_out/trace_writers.log; exit $rc
