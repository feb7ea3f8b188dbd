# HBM traffic of the pipelined kernel from PMC counters (run via gpurun):
# one FETCH_SIZE pass and one WRITE_SIZE pass over the bench workload, each
# counter in its own run as MI355X_MICROARCH.md (rocprofv3 PMC slots) requires.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c -d $GRAFT_REPO_ROOT/gpurun_out/pmc_$c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 12 --warmup 0 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/pmc_$c.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/pmc_WRITE_SIZE/run_counter_collection.csv > gpurun_out/pmc_traffic.json
cat gpurun_out/pmc_traffic.json
