#!/bin/bash
# Round-4 batch 3: per-block cycle anatomy of the persistent forward (base and prescaled).
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/asm_pstamps.py > gpurun_out/pstamps_r04.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/asm_pstamps.py --gen "--prescale 1 --kfirst 2 --xphase 1" >> gpurun_out/pstamps_r04.txt 2>&1
