set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for hop in 6 10 14 18 26; do
  HL_AMD_PIPE_HOP=$hop timeout -k 10 300 python -u bench.py --svc --no-cpu-baseline > gpurun_out/svchop_$hop.log 2>&1 || { tail -5 gpurun_out/svchop_$hop.log; exit 1; }
  echo "hop $hop: $(grep -o '"value": [0-9.]*' gpurun_out/svchop_$hop.log | head -1) $(grep -o '"bitexact": [a-z]*' gpurun_out/svchop_$hop.log)"
done
