# SVC GPU tests + config-4 bench (one GPU, and a 3-rank gloo rehearsal)
set -o pipefail
tag=${1:-svc}
bash tools/gpu_svc.sh && bash tools/gpu_svc_bench.sh $tag
