#!/bin/bash
# Generator options re-checked on the persistent forward (north star, one process, interleaved).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/asm_variants.py --rounds 7 --variants "p:--persist 1;dmap2:--persist 1 --dmap2 1;vp0:--persist 1 --vp1 0;lag33:--persist 1 --lag 3,3;lag54:--persist 1 --lag 5,4;lag45:--persist 1 --lag 4,5" > gpurun_out/persist_opts.txt 2>&1
