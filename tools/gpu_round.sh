set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r01_final_tests.log 2>&1 || { tail -30 gpurun_out/r01_final_tests.log; exit 1; }
tail -3 gpurun_out/r01_final_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r01_final_bench.log 2>&1 || { tail -30 gpurun_out/r01_final_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r01_final_bench.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py > gpurun_out/r01_final_prof.log 2>&1 || { tail -30 gpurun_out/r01_final_prof.log; exit 1; }
tail -2 gpurun_out/r01_final_prof.log
