#!/bin/bash
# A/B of the persistent asm forward (gen_fwd.py --persist 1: next-Q prefetch) against the shipped
# one-block-per-workgroup form; correctness check of each against torch fp32 on sequence 0.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --rounds 7 --variants ";persist:--persist 1;nopro:--probe nopro" > gpurun_out/persist_ab.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --shape 16,12,2048 --rounds 5 --variants ";persist:--persist 1" >> gpurun_out/persist_ab.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --shape 4,16,4096 --rounds 5 --variants ";persist:--persist 1" >> gpurun_out/persist_ab.txt 2>&1
