set -u
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h/pytest_gpu.txt 2>&1 || exit $?
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 120 python3 scripts/step_probe.py --rounds 2 --opt 38=$v --json gpurun_out/r6h/step${v}_$r.json > gpurun_out/r6h/step${v}_$r.out 2>&1 || exit $?
  done
done
