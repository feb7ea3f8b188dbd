#!/bin/bash
# Diagnosis of the pipelined-run mismatch on the GPU box: the
# GOP-spanning stress run on the round-1 build (build/old) and on the same
# build with the per-step candidate results double-buffered (build/oldC).
set -o pipefail
mkdir -p gpurun_out
run() {  # name, seconds, command...
    local name=$1 secs=$2
    shift 2
    echo "== $name"
    timeout -k 10 "$secs" "$@" > "gpurun_out/diag_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(tail -1 gpurun_out/diag_$name.log)"
    case $rc in 124|134|137|139) exit $rc ;; esac
    return 0
}
S="python -u tools/stress_spans_gops.py"
for v in old oldC old oldC old oldC; do
    HL_LIB=build/$v/libhartallo_amd.so run stress_$v 200 $S 8
done
run stress_new 200 $S 8
