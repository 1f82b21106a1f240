#!/bin/bash
# Round-4: head dims between the asm tiles (80, 96: HIP kernels) against D=128 (asm), fwd and bwd.
mkdir -p gpurun_out
rm -f gpurun_out/dpad_r04.txt
for c in D64 D80 D96 D128; do for m in fwd bwd; do
  timeout -k 10 120 python tools/tiles_run.py --cfg $c --mode $m --launches 100 >> gpurun_out/dpad_r04.txt 2>&1 || exit 1
done; done
