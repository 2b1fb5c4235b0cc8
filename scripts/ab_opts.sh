# A/B of bench flags on the product library: OPTS="label1:flags1;label2:flags2" ARGS="common flags"
# -> gpurun_out/ab_<label>_<k>.json (summarise with scripts/ab_summary.py label1 label2)
set -e
cd "${GRAFT_REPO_ROOT}"
IFS=';' read -ra SETS <<< "${OPTS}"
for k in 1 2; do
  for s in "${SETS[@]}"; do
    lab=${s%%:*}; fl=${s#*:}
    timeout -k 10 200 python bench.py --no-cpu-baseline --loop-epochs 0 ${ARGS} $fl > gpurun_out/ab_${lab}_$k.json
  done
done
echo ok
