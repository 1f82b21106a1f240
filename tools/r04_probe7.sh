#!/bin/bash
# Round-4: rescale-test placement (gen_fwd --ptail N: test before the phase's last N MFMAs).
mkdir -p gpurun_out
rm -f gpurun_out/pstamps_r04q.txt
for v in "" "--qlate 0"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> gpurun_out/pstamps_r04q.txt 2>&1 || exit 1
done
