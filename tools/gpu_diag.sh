#!/bin/bash
# Diagnosis of the pipelined-run mismatch, run on the GPU box
# from the repo root: the GOP-spanning stress run on the input-digest build
# (HL_DIAG_INPUTS: each record carries digests of the MB's inputs, so a
# mismatch names the first input that differed).
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
HL_LIB=build/dinp/libhartallo_amd.so run stress_dinp 300 $S 10
