# A/B probe runs on the GPU box: per-kernel µs of one layer (C3 survey + relcond), forward and training step
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in fb15k237 fb15k237_relcond; do
  timeout -k 10 120 python scripts/layer_ab.py --workload $w --label "$w" >> gpurun_out/ab.jsonl
  timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd" >> gpurun_out/ab.jsonl
  MPGNN_OUTER_OLD=1 timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd-oldouter" >> gpurun_out/ab.jsonl
done
cat gpurun_out/ab.jsonl
