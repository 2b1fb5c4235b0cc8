set -u
mkdir -p gpurun_out/r6pad
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "outer_variants" > gpurun_out/r6pad/t.txt 2>&1 || exit $?
timeout -k 10 300 python3 scripts/ab_opt_layer.py --opt 38 --values 0,1 --iters 30 --rounds 3 > gpurun_out/r6pad/ab_pad.json 2> gpurun_out/r6pad/ab_pad.err || exit $?
timeout -k 10 200 python3 scripts/step_probe.py --opt 38=0 --json gpurun_out/r6pad/step0.json > gpurun_out/r6pad/step0.out 2>&1 || exit $?
timeout -k 10 200 python3 scripts/step_probe.py --opt 38=1 --json gpurun_out/r6pad/step1.json > gpurun_out/r6pad/step1.out 2>&1 || exit $?
