# GPU pass of a candidate change: the GPU unit / parity / pipeline tests on
# the in-tree product, then tools/ab_bench.py on the listed builds.
#   bash tools/gpu_ab.sh tag lib1.so [lib2.so ...]
set -o pipefail
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_unit.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_bench_golden.py > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/ab_bench.py "$@" > gpurun_out/${tag}_ab.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/${tag}_ab.log; exit $rc
