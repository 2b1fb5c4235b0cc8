#!/bin/bash
# Upper bound of overlapping the segment means with the transform GEMM: probe
# libraries (-DMPGNN_PROBE_OVERLAP=1|2, WRONG results: the GEMM reads stale means) that launch the
# means on a side stream concurrently with the GEMM; the C3 forward step (scripts/step_probe.py)
# with the product library and both probes, alternated three times in fresh processes.
# Build here (CPU): bash scripts/r06_probe_overlap.sh build ; then on the box: bash scripts/r06_probe_overlap.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [[ ${1:-} == build ]]; then
  cd mpgnn-metapath-graph-neural-network_amd/csrc
  for v in 1 2; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -ffp-contract=off \
        -DMPGNN_PROBE_OVERLAP=$v -I../../include -I. -shared -o ../libmpgnn_rgcn_probe$v.so \
        plan.cpp io.cpp rgcn_kernels.hip plan_device.hip score_kernels.hip &
  done
  wait
  exit 0
fi
O=${O:-gpurun_out/r6ov}
mkdir -p $O
L=$PWD/mpgnn-metapath-graph-neural-network_amd
for r in 1 2 3; do
  timeout -k 10 120 python3 scripts/step_probe.py --rounds 2 --json $O/prod_$r.json > $O/prod_$r.out 2>&1 || exit $?
  for v in 1 2; do
    MPGNN_LIB_PATH=$L/libmpgnn_rgcn_probe$v.so timeout -k 10 120 python3 scripts/step_probe.py --rounds 2 --no-check \
        --json $O/probe${v}_$r.json > $O/probe${v}_$r.out 2>&1 || exit $?
  done
done
echo done
