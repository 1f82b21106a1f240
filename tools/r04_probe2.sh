#!/bin/bash
# Round-4 batch 2: per-block fixed cost fit (one-block vs persistent), and the K-first / cross-phase
# lgkmcnt / prescaled-Q variants of the persistent D=64 forward (one process, interleaved).
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/asm_variants.py --rounds 5 --variants \
  "base:--persist 1;kx:--persist 1 --kfirst 2 --xphase 1;ps:--persist 1 --prescale 1;pskx:--persist 1 --prescale 1 --kfirst 2 --xphase 1;x:--persist 1 --xphase 1" \
  > gpurun_out/var_r04b.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/fixed_cost_fit.py > gpurun_out/fixed_fit_r04.txt 2>&1
