#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no trace domains) of the north-star forward in
# several (library, impl) legs, for the issue / co-execution comparison of the 4-wave and the
# staggered 8-wave forms (tools only):
#   bash tools/r05/forms_pmc.sh <outdir> "<lib:impl> ..."     (lib "prod" = the product library)
set -e
OUT=$1; LEGS=$2
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for leg in $LEGS; do
  lib=${leg%%:*}; impl=${leg##*:}; i=0
  if [ "$lib" = prod ]; then unset FA_HIP_LIB; else export FA_HIP_LIB=$L/libfa_hip_$lib.so; fi
  for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
             "SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    mkdir -p "$OUT/$lib-$impl"
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/$lib-$impl/p$i" -o p --output-format csv -- \
      python tools/tiles_run.py --cfg D64 --mode fwd --launches 5 --warm 0.05 --impl $impl > "$OUT/$lib-$impl/p$i.log" 2>&1
  done
done
