set -u
mkdir -p gpurun_out/r6u
timeout -k 10 300 python3 scripts/ab_opt_layer.py --opt 37 --values 16,32,8 --iters 30 --rounds 3 > gpurun_out/r6u/ab_u.json 2> gpurun_out/r6u/ab_u.err || exit $?
