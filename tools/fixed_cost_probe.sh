#!/bin/bash
# Price of the per-workgroup prologue burst (Q loads + first K/V DMAs) and epilogue store tail of the
# D=64 asm forward at the north star: timing probes (wrong results by design), one process.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --rounds 7 --variants ";nopro:--probe nopro;noepi:--probe noepi;both:--probe nopro,noepi" > gpurun_out/fixed_cost.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --shape 16,12,2048 --rounds 5 --variants ";nopro:--probe nopro;noepi:--probe noepi" >> gpurun_out/fixed_cost.txt 2>&1
