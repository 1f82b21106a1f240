#!/bin/bash
# D=128: tile-end waits sized to the pieces per tile (16) against the stricter round-3 count (8);
# D=32: correctness and time of the fixed one-block tile (and the persistent one) vs the HIP kernel.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --hd 128 --rounds 7 --variants ";strict:--probe strictwait" > gpurun_out/wait_ab.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --hd 32 --rounds 7 --variants ";persist:--persist 1" >> gpurun_out/wait_ab.txt 2>&1
