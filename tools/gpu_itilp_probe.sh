# GPU-box: which pipelined-run parity tests the iterative-ilp build (build/var/itilp.so) fails (box-local copy over the product library).
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
cp build/var/itilp.so hartallo_amd/libhartallo_amd.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -v --timeout 200 --timeout-method thread > gpurun_out/itilp_probe.log 2>&1
grep -E "PASSED|FAILED|first differing|passed|failed" gpurun_out/itilp_probe.log | grep -v "^E  .*assert b" | head -40
exit 0
