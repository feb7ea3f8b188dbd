#!/bin/bash
# Builds the product library of a git revision into build/<name>/ (A/B
# baselines for tools/ab_bench.py).  Development tool, build container:
#   bash tools/build_rev.sh REV NAME [extra hipcc flags]
set -e
rev=$1; name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" hartallo_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/build/$name"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable \
    -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" -shared -o "$root/build/$name/libhartallo_amd.so" \
    "$tmp"/hartallo_amd/csrc/hl_encoder.hip "$tmp"/hartallo_amd/csrc/hl_encoder_fam3.hip "$tmp"/hartallo_amd/csrc/hl_writer.cpp "$tmp"/hartallo_amd/csrc/hl_rc.cpp 2>&1 | grep -v warning | grep -i error || true
rm -rf "$tmp"
ls -la "$root/build/$name/libhartallo_amd.so"
