#!/bin/bash
# A/B of the persistent D=128 asm forward (K/V tail only) against the one-block form.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --hd 128 --rounds 7 --variants ";persist:--persist 1" > gpurun_out/persist128_ab.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --hd 128 --shape 16,12,4096 --rounds 5 --variants ";persist:--persist 1" >> gpurun_out/persist128_ab.txt 2>&1
