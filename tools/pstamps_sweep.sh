#!/bin/bash
# Per-block cycle anatomy of generator variants of the persistent D=64 forward (tools/asm_pstamps.py,
# one variant per process, same box): prologue / loop per tile / last tile + epilogue / seam.
#   bash tools/pstamps_sweep.sh <out.txt> "" "--ksplit 2" "--probe nobar" ...
# ("" = the product settings; --probe switches give wrong results by design, timing only)
OUT=${1:-gpurun_out/pstamps.txt}
shift
mkdir -p "$(dirname "$OUT")"
rm -f "$OUT"
for v in "$@"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> "$OUT" 2>&1 || exit 1
done
