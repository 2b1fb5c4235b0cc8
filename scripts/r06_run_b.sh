set -u
mkdir -p gpurun_out/r6o
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "outer_variants" > gpurun_out/r6o/t.txt 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_opt_layer.py --opt 36 --values 0,2,1 --iters 30 --rounds 3 > gpurun_out/r6o/ab_var.json 2> gpurun_out/r6o/ab_var.err || exit $?
