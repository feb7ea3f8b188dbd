# GPU-box: smoke() on cuda:0, then the rocprofv3 kernel-stats summary (csv) of the default bench command.
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r01_smoke.log 2>&1 || { tail -20 gpurun_out/r01_smoke.log; exit 1; }
tail -2 gpurun_out/r01_smoke.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_final -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py > gpurun_out/r01_final_prof.log 2>&1 || { tail -30 gpurun_out/r01_final_prof.log; exit 1; }
grep '"metric"' gpurun_out/r01_final_prof.log
