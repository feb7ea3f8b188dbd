# Round-end style GPU check (run via gpurun from the repo root):
# all -m gpu tests, the default bench, and a rocprofv3 kernel trace of a
# short bench whose summary goes under gpurun_out/prof.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
cat $(find gpurun_out/prof -name "*kernel_stats.csv" | head -1) | cut -c1-200
