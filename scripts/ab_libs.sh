# A/B of library builds (mpgnn-metapath-graph-neural-network_amd/lib<tag>.so) on the C3 bench:
# usage: TAGS="v1 v2" ARGS="..." bash scripts/ab_libs.sh   (outputs gpurun_out/ab_<tag>_<k>.json)
set -e
cd "${GRAFT_REPO_ROOT}"
D=$PWD/mpgnn-metapath-graph-neural-network_amd
for k in 1 2; do
  for t in base ${TAGS}; do
    if [ "$t" = base ]; then L=$D/libmpgnn_rgcn.so; else L=$D/lib$t.so; fi
    MPGNN_LIB_PATH=$L MPGNN_ALLOW_STALE_LIB=1 timeout -k 10 150 python bench.py --no-cpu-baseline --loop-epochs 0 ${ARGS} > gpurun_out/ab_${t}_$k.json
  done
done
echo ok
