#!/bin/bash
# GPU check of the asm forward after a change: the whole -m gpu suite, then event-time A/B of the
# asm kernels against the HIP ones (FaFwdArgs.impl) on the BASELINE-like shapes they serve.
set -e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_asm.txt 2>&1
for r in 1 2; do for c in C3nd C4 D128b16 D64 D128; do for i in auto hip; do
  timeout -k 10 120 python tools/tiles_r03.py --cfg $c --mode fwd --launches 100 --impl $i >> gpurun_out/asm_time.txt 2>&1
done; done; done
