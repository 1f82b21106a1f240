#!/bin/bash
# Fixed cost per workgroup of the asm forward: non-causal C4 grids (B16 H12 Sq4096 D128) with
# Sk = 256..4096 (4..64 tiles per workgroup), fit time = a * workgroups/CU + b * tiles/CU.
set -e
for sk in 256 512 1024 2048 4096; do
  timeout -k 10 120 python tools/tiles_r03.py --cfg 16,12,4096,$sk,128 --mode fwd --launches 50 >> gpurun_out/wg_overhead.txt 2>/dev/null
  timeout -k 10 120 python tools/tiles_r03.py --cfg 16,12,4096,$sk,64 --mode fwd --launches 50 >> gpurun_out/wg_overhead.txt 2>/dev/null
done
timeout -k 10 120 python tools/tiles_r03.py --cfg C4 --mode fwd --launches 50 >> gpurun_out/wg_overhead.txt 2>/dev/null
