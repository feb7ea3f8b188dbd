# GPU-box: pipelined-run parity (incl. GOP-spanning 1088p batches), a stress repeat of that batch, then the bench.
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || { tail -30 gpurun_out/split_tests.log; exit 1; }
tail -1 gpurun_out/split_tests.log
timeout -k 10 200 python -u tools/stress_spans_gops.py 8 > gpurun_out/split_stress.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/split_stress.log | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/split_bench.log 2>&1 || { tail -30 gpurun_out/split_bench.log; exit 1; }
grep '"metric"' gpurun_out/split_bench.log
