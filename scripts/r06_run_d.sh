set -u
mkdir -p gpurun_out/r6s
timeout -k 10 200 python3 scripts/stamps_gemm_il.py --opt 35=1 > gpurun_out/r6s/w1.json 2> gpurun_out/r6s/w1.err || exit $?
timeout -k 10 200 python3 scripts/stamps_gemm_il.py > gpurun_out/r6s/bf3.json 2> gpurun_out/r6s/bf3.err || exit $?
