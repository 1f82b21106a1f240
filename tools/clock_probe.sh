#!/bin/bash
# Effective shader clock and MFMA-pipe utilisation of one variant library on the north-star shape:
#   bash tools/clock_probe.sh <variant> <outdir>     (FA_VARIANTS must define the variant)
# clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time; MFMA util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
set -e
V=$1; OUT=$2
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
FA_CONFIGS=ns timeout -k 10 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d "$OUT" -o p --output-format csv -- python tools/fwd_variants.py run --only "$V" --rounds 2 --iters 10 > "$OUT.log" 2>&1
