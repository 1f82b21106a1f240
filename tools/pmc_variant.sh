#!/bin/bash
# PMC passes over one asm-forward generator variant (tools/asm_variants.py, one variant per process so
# the kernel name is unambiguous); one rocprofv3 run per counter group, no trace domains.
#   bash tools/pmc_variant.sh <outdir> "<generator args>"
set -e
OUT=$1; ARGS=$2
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"; i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INST_LEVEL_LDS" \
           "SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_EXP SQ_INST_CYCLES_VMEM SQ_INSTS_SMEM SQ_IFETCH SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o p --output-format csv -- \
      python tools/asm_variants.py --variants "v:$ARGS" --rounds 1 --iters 10 > "$OUT/p$i.log" 2>&1 || echo "pass $i failed" >> "$OUT/fail.txt"
done
