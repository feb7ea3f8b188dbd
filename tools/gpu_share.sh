#!/bin/bash
# Streams sharing one GPU: bench.py's driver workload (--steps 20 --warmup 5)
# with 1, 2 and 4 ranks on the box's one GPU (each rank its own stream and its
# share of the CUs).  GPU box, repo root:  bash tools/gpu_share.sh [steps]
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
steps=${1:-20}
for n in ${NS:-1 2 4}; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
      bench.py --gpus $n --steps $steps --warmup 5 --no-cpu-baseline > gpurun_out/share_$n.log 2>&1 || { tail -5 gpurun_out/share_$n.log; exit 1; }
  grep '^{' gpurun_out/share_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, 'ranks:', d['value'], 'fps total, bitexact', d['bitexact'], d['pipeline'])"
done
