#!/bin/bash
# Second pass: reordered, with the combination (north star and B16).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/asm_variants.py --rounds 9 --variants "vp0lag33:--persist 1 --vp1 0 --lag 3,3;lag33:--persist 1 --lag 3,3;p:--persist 1;vp0:--persist 1 --vp1 0" > gpurun_out/persist_opts2.txt 2>&1
timeout -k 10 300 python -u tools/asm_variants.py --shape 16,12,2048 --rounds 5 --variants "vp0:--persist 1 --vp1 0;p:--persist 1;vp0lag33:--persist 1 --vp1 0 --lag 3,3;lag33:--persist 1 --lag 3,3" >> gpurun_out/persist_opts2.txt 2>&1
