#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only — no sys/runtime trace)
# over scripts/prof_layer.py; summaries: python scripts/pmc_summary.py gpurun_out/pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc}
mkdir -p "$OUT"
ARGS=${ARGS:---iters 20}
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
    i=$((i+1))
    echo "== pass $i: $grp"
    timeout -k 10 300 rocprofv3 --pmc $grp -d "$OUT/p$i" -o run --output-format csv -- python3 scripts/prof_layer.py $ARGS > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "rc=$rc"
    case $rc in 0) ;; *) echo "pass $i failed, stopping"; tail -5 "$OUT/p$i.log"; exit $rc;; esac
done
