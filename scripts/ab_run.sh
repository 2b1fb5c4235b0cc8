# A/B probe runs on the GPU box: per-kernel µs of one layer's training step — the product
# library vs the previous build (MPGNN_LIB_PATH=libmpgnn_old.so)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$PWD/mpgnn-metapath-graph-neural-network_amd/libmpgnn_old.so
for w in fb15k237 C2; do
  for k in 1 2; do
    timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-new" >> gpurun_out/ab.jsonl
    MPGNN_LIB_PATH=$V MPGNN_ALLOW_STALE_LIB=1 timeout -k 10 120 python scripts/layer_ab.py --workload $w --backward --label "$w-old" >> gpurun_out/ab.jsonl
  done
done
cat gpurun_out/ab.jsonl
