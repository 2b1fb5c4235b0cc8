# prologue records on by default: the GPU suite
set -u
O=${O:-gpurun_out/r6ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/t_all.txt 2>&1 || exit $?
