#!/bin/bash
# Part 2 of the round-3 evidence plus the workgroup fixed-cost probes of the asm forward.
set -e
bash tools/round3_final.sh 2
timeout -k 10 120 python -u tools/asm_wg_timeline.py > gpurun_out/wg_timeline.txt 2>&1
bash tools/asm_wg_overhead.sh
