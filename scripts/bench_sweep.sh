# every workload's bench line (1 GPU) -> gpurun_out/sweep/<tag>.json; SET=a|b splits the sweep
set -e
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sweep
run() { tag=$1; shift; timeout -k 10 ${T:-400} python bench.py "$@" > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err; }
if [ "${SET:-a}" = a ]; then
  run c3_relcond --workload fb15k237_relcond
  run c2 --workload C2
  run c2_single --workload C2 --mode single
  run c3_score --mode score
else
  T=560 run c5 --workload C5
  T=500 run c5_single --workload C5 --mode single
fi
echo ok
