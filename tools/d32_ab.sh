#!/bin/bash
# The D=32 asm tile (one-block and persistent) against the HIP D=32 forward, B8 H12 S2048.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --hd 32 --rounds 7 --variants ";persist:--persist 1" > gpurun_out/d32_ab.txt 2>&1
for i in 1 2 3; do timeout -k 10 120 python tools/tiles_r03.py --cfg D32 --mode fwd --launches 100 --impl hip >> gpurun_out/d32_ab.txt 2>/dev/null; done
