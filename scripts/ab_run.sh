# A/B probe runs on the GPU box: per-kernel µs of one C3 layer, forward and training step
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lab in ${AB_LABELS:-cur}; do
  timeout -k 10 120 python scripts/layer_ab.py --label "$lab" >> gpurun_out/ab.jsonl
  timeout -k 10 120 python scripts/layer_ab.py --backward --label "$lab-bwd" >> gpurun_out/ab.jsonl
done
cat gpurun_out/ab.jsonl
