# SVC tests, then bench.py --svc under chunk:pipeline-workgroup settings
#   CFGS="8:0 31:128" NOTEST=1 bash tools/gpu_svc_sweep.sh <tag>
set -o pipefail
tag=${1:-sweep}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$NOTEST" ] || bash tools/gpu_svc.sh || exit 1
for cfg in ${CFGS:-8:0 31:0}; do
    c=${cfg%%:*}; w=${cfg##*:}
    HL_AMD_SVC_CHUNK=$c HL_AMD_PIPE_WG=$w timeout -k 10 300 python -u bench.py --svc > gpurun_out/${tag}_c${c}_w${w}.log 2>&1 || { tail -20 gpurun_out/${tag}_c${c}_w${w}.log; exit 1; }
    echo "chunk $c wg $w: $(grep -o '"value": [0-9.]*' gpurun_out/${tag}_c${c}_w${w}.log | head -1) $(grep -o '"bitexact": [a-z]*' gpurun_out/${tag}_c${c}_w${w}.log)"
done
