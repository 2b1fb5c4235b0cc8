set -u
mkdir -p gpurun_out/r6e
timeout -k 10 300 python3 scripts/ab_opt_layer.py --opt 29 --values 250,100,400,0 --iters 30 --rounds 3 > gpurun_out/r6e/ab_switch.json 2> gpurun_out/r6e/ab_switch.err || exit $?
timeout -k 10 300 python3 scripts/ab_opt_layer.py --opt 26 --values 0,2,4 --iters 30 --rounds 3 > gpurun_out/r6e/ab_wgcu.json 2> gpurun_out/r6e/ab_wgcu.err || exit $?
