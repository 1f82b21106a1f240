#!/bin/bash
# Per-tile roofline evidence (profiles/r0N_tiles_roofline.json; round 4 adds D80 and D96):
# for each configuration and mode (forward-only loop, backward-only loop) one steady-state
# kernel-trace pass (>= 0.3 s warm-up, then 200 timed calls, event time printed by the driver)
# and three short PMC passes (FETCH_SIZE; WRITE_SIZE; MFMA busy + GRBM + MFMA/VALU instruction
# counts). Counter passes never combine with other trace domains.
#   bash tools/tiles.sh <outdir> [cfg ...]        (default: D32 D64 D128 C2 C3 C4 C5)
set -e
OUT=${1:-gpurun_out/tiles}
shift || true
CFGS=${*:-D32 D64 D128 C2 C3 C4 C5}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for c in $CFGS; do
  for m in fwd bwd; do
    P="python tools/tiles_run.py --cfg $c --mode $m"
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/$c.$m/trace" -o t --output-format csv -- $P --launches 200 > "$OUT/$c.$m.trace.log" 2>&1
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/$c.$m/fetch" -o p --output-format csv -- $P --launches 10 --warm 0.05 > "$OUT/$c.$m.fetch.log" 2>&1
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/$c.$m/write" -o p --output-format csv -- $P --launches 10 --warm 0.05 > "$OUT/$c.$m.write.log" 2>&1
    timeout -k 10 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU -d "$OUT/$c.$m/mfma" -o p --output-format csv -- $P --launches 10 --warm 0.05 > "$OUT/$c.$m.mfma.log" 2>&1
    echo "$c $m done"
  done
done
