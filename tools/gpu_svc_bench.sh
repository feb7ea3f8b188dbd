# Config-4 (spatial SVC) bench on one GPU box: all layers on one GPU, a
# 2-rank streams rehearsal (two ranks share the one GPU, one stream each) and
# a 3-rank layer-sharded rehearsal with gloo (three ranks share the one GPU;
# RCCL needs one GPU per rank).  bash tools/gpu_svc_bench.sh <tag>
set -o pipefail
tag=${1:-svc}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --svc > gpurun_out/${tag}_bench1.log 2>&1 || { tail -20 gpurun_out/${tag}_bench1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_bench1.log | tail -1
HL_SVC_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --svc > gpurun_out/${tag}_bench2_streams.log 2>&1 || { tail -30 gpurun_out/${tag}_bench2_streams.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_bench2_streams.log | grep metric | tail -1
HL_SVC_SHARD=layers HL_SVC_BACKEND=gloo timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29533 bench.py --svc > gpurun_out/${tag}_bench3_gloo.log 2>&1 || { tail -30 gpurun_out/${tag}_bench3_gloo.log; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_bench3_gloo.log | grep metric | tail -1
