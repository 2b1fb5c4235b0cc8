# A/B probe runs on the GPU box: per-kernel µs of one C3 layer's training step (backward
# weight-gradient chunk length sweep)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cr in 224 256 288 320 256 224; do
  timeout -k 10 120 python scripts/layer_ab.py --workload fb15k237 --backward --chunk-rows $cr --label "bwd-cr$cr" >> gpurun_out/ab.jsonl
done
cat gpurun_out/ab.jsonl
