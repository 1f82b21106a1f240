#!/bin/bash
# Round-4: loop cycle anatomy of the product forward (prescaled bf16, K-first, cross-phase waits):
# per-block stamps of the product and of timing probes (wrong results by design), cycles per tile.
mkdir -p gpurun_out
rm -f gpurun_out/pstamps_r04b.txt
for v in "" "--probe noor" "--probe nolds" "--probe nodma" "--probe nobar" "--probe nosum" "--probe nocvt" "--probe noexp" "--vp1 0" "--lag 4,2" "--lag 4,6"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> gpurun_out/pstamps_r04b.txt 2>&1 || exit 1
done
