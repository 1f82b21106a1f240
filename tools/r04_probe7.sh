#!/bin/bash
# Round-4: rescale-test placement (gen_fwd --ptail N: test before the phase's last N MFMAs).
mkdir -p gpurun_out
rm -f gpurun_out/pstamps_r04p.txt
for v in "" "--kvtail 0" "--kvtail 0 --ring 6 --dist 4" "--kvtail 0 --ring 6 --dist 4 --bar2 1"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> gpurun_out/pstamps_r04p.txt 2>&1 || exit 1
done
