set -e
cd "${GRAFT_REPO_ROOT}"
V=$PWD/mpgnn-metapath-graph-neural-network_amd/libmpgnn_old.so
for k in 1 2; do
  timeout -k 10 150 python bench.py --mode single --workload fb15k237 --no-cpu-baseline --epoch-steps 10 > gpurun_out/s_new_$k.json
  MPGNN_LIB_PATH=$V MPGNN_ALLOW_STALE_LIB=1 timeout -k 10 150 python bench.py --mode single --workload fb15k237 --no-cpu-baseline --epoch-steps 10 > gpurun_out/s_old_$k.json
done
