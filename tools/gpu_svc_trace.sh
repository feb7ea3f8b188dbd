# kernel trace of bench.py --svc (timestamps: do the enhancement layers overlap the base runs?)
set -o pipefail
tag=${1:-svctrace}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
HL_AMD_SVC_CHUNK=${2:-8} HL_AMD_PIPE_WG=${3:-0} timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${tag} -o run --output-format csv -- python3 bench.py --svc > gpurun_out/${tag}.log 2>&1 || { tail -20 gpurun_out/${tag}.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/${tag}.log
