#!/bin/bash
# Upper bound of what pre-split bf16 operand planes could save: a probe
# library whose split3_bf16 keeps only the first piece (-DMPGNN_PROBE_NOSPLIT: same loads, LDS
# traffic and MFMA count, no split VALU, WRONG results) A/B'd against the product library on one
# box with scripts/r05_ab_lib_c3.sh (it loads the probe as libmpgnn_rgcn_prev.so).
# Build here (CPU), then: gpurun -- 'OUT=gpurun_out/r6b bash scripts/r05_ab_lib_c3.sh'
set -e
cd "$(dirname "$0")/../mpgnn-metapath-graph-neural-network_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -Wall -Wno-unused-function --offload-arch=gfx950 -ffp-contract=off \
    -DMPGNN_PROBE_NOSPLIT -I../../include -I. -shared -o ../libmpgnn_rgcn_prev.so \
    plan.cpp io.cpp rgcn_kernels.hip plan_device.hip score_kernels.hip
