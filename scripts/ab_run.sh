# A/B probe runs on the GPU box: per-kernel µs of one C3 layer's training step, env switches
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in fb15k237; do
  timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd" >> gpurun_out/ab.jsonl
  MPGNN_OUTER_SL32=1 timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd-sl32" >> gpurun_out/ab.jsonl
  timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd" >> gpurun_out/ab.jsonl
  MPGNN_OUTER_SL32=1 timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-bwd-sl32" >> gpurun_out/ab.jsonl
done
cat gpurun_out/ab.jsonl
