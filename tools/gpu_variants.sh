# GPU-box: time compiler-flag variants of the library (build/var/*.so) and run geometries on a pipelined run of 60 P pictures.
set -o pipefail
mkdir -p gpurun_out
cd $GRAFT_REPO_ROOT
for v in itilp itmin itocc itilp; do
  echo "== $v"
  HL_LIB=build/var/$v.so timeout -k 10 120 python -u tools/pipe_bench.py 60 > gpurun_out/var_$v.log 2>&1 || { tail -20 gpurun_out/var_$v.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/var_$v.log | tail -3
done
echo "== itilp geometries"
HL_LIB=build/var/itilp.so timeout -k 10 200 python -u tools/pipe_bench.py 60 0,1,64 0,3,64 0,2,16 512,2,64 > gpurun_out/var_geo.log 2>&1 || { tail -20 gpurun_out/var_geo.log; exit 1; }
grep -v amdgpu.ids gpurun_out/var_geo.log | tail -5
