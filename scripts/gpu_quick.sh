# quick GPU check: a pytest -k selection ($K), then bench lines ($BENCH: ';'-separated arg sets) -> gpurun_out/quick
set -e
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/quick
if [ -n "${K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/quick/tests.log 2>&1
fi
i=0
IFS=';' read -ra SETS <<< "${BENCH:-}"
for a in "${SETS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py $a > gpurun_out/quick/bench_$i.json 2> gpurun_out/quick/bench_$i.err
done
echo ok
