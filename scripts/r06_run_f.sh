set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r6st
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r6st/w8 -o run --output-format csv -- python3 scripts/shard_trace.py 8 3 > gpurun_out/r6st/w8.out 2>&1 || exit $?
