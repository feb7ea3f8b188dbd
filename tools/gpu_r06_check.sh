#!/bin/bash
# Round 6: op-level parity (tests/test_gpu_ops.py) and the new golden cases
# (QP 4's 2^30 lambda, the QP 8 reference failure, max_ref_frame above 16)
# on the GPU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
    tests/test_gpu_parity.py -k "ops or reference or qp4 or fails or mrf" > gpurun_out/r06_check.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/r06_check.log | tail -40; exit $rc
