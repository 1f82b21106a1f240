#!/bin/bash
# Per-head-dim-tile roofline evidence (BASELINE north star: "rocprof must show the achieved MFMA
# utilisation and HBM GB/s ... for each head-dim tile"). For D in 32/64/128 at B=8 H=12 S=2048,
# non-causal, forward + backward: one kernel-trace/stats pass and three PMC passes (FETCH_SIZE,
# WRITE_SIZE, MFMA busy). Counter passes never combine with trace domains.
#   bash tools/profile_tiles.sh <outdir>
set -e
OUT=${1:-gpurun_out/tiles}
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
for D in 32 64 128; do
  [ -n "$TRACE_ONLY" ] && { timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/d$D/trace" -o t --output-format csv -- python tools/run_fwd.py --B 8 --H 12 --S 2048 --D $D --iters 60 --bwd 1 > "$OUT/d$D.trace.log" 2>&1; continue; }
  A="--B 8 --H 12 --S 2048 --D $D --iters 5 --bwd 1"
  # the timing pass runs long enough for the clock to ramp (tiles_summary drops the first fifth)
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/d$D/trace" -o t --output-format csv -- python tools/run_fwd.py --B 8 --H 12 --S 2048 --D $D --iters 60 --bwd 1 > "$OUT/d$D.trace.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/d$D/fetch" -o p --output-format csv -- python tools/run_fwd.py $A > "$OUT/d$D.fetch.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/d$D/write" -o p --output-format csv -- python tools/run_fwd.py $A > "$OUT/d$D.write.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA -d "$OUT/d$D/mfma" -o p --output-format csv -- python tools/run_fwd.py $A > "$OUT/d$D.mfma.log" 2>&1
done
