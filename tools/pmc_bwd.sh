#!/bin/bash
# PMC passes over the backward of one configuration (separate rocprofv3 runs per counter group).
#   bash tools/pmc_bwd.sh <outdir> [run_fwd.py args...]
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"; i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p --output-format csv -- python tools/run_fwd.py --iters 3 --bwd 1 "$@" > "$OUT/p$i.log" 2>&1
done
