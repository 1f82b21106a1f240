#!/bin/bash
# Round-4: rescale-test placement (gen_fwd --ptail N: test before the phase's last N MFMAs).
mkdir -p gpurun_out
rm -f gpurun_out/pstamps_r04m.txt
for v in "--ksplit 1" "--ksplit 2" "--ksplit 3" "--ksplit 2 --ptail 2"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> gpurun_out/pstamps_r04m.txt 2>&1 || exit 1
done
