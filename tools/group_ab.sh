#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/asm_group_ab.py --groups 0,1,2,3,4,6 > gpurun_out/group_ab.txt 2>&1
timeout -k 10 300 python -u tools/asm_group_ab.py --hd 64 --shape 8,12,2048 --groups 0,1,2,3,4 >> gpurun_out/group_ab.txt 2>&1
