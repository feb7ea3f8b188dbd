set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_svc.py -x -v --timeout 300 --timeout-method thread > gpurun_out/svc_tests.log 2>&1
rc=$?
tail -15 gpurun_out/svc_tests.log
exit $rc
