#!/bin/bash
# Round 6: FETCH_SIZE / WRITE_SIZE calibration for the kernel's access
# patterns (tools/fetch_calib.hip, built in-tree as build/fetch_calib): one
# counter set per rocprofv3 pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fcal2
i=0
for set in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "WRITE_SIZE" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/fcal2/p$i -o run --output-format csv -- build/fetch_calib > gpurun_out/fcal2/p$i.log 2>&1 || exit $?
done
grep '^{' gpurun_out/fcal2/p1.log
python3 tools/fetch_calib_summary.py gpurun_out/fcal2/p*/run_counter_collection.csv
