#!/bin/bash
# A/B of the two-waves-per-SIMD assembly forward (gen_fwd.py --waves 8) against the one-wave form,
# with a correctness check of each against torch fp32 on sequence 0, then the -m gpu suite.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/asm_variants.py --variants ";w8:--waves 8" --rounds 7 > gpurun_out/w8_ab.txt 2>&1
timeout -k 10 200 python -u tools/asm_variants.py --shape 16,12,2048 --variants ";w8:--waves 8" --rounds 5 >> gpurun_out/w8_ab.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_w8.txt 2>&1
