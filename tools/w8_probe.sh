#!/bin/bash
# Anatomy of the two-waves-per-SIMD forward: timing probes (wrong results by design) and options.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/asm_variants.py --rounds 5 --variants ";w8:--waves 8;w8p:--waves 8 --prio4 1;w8nofill:--waves 8 --probe nofill;w8nolds:--waves 8 --probe nolds;w8nodma:--waves 8 --probe nodma;w8nobar:--waves 8 --probe nobar;w8nomfma:--waves 8 --probe nomfma;w8noexp:--waves 8 --probe noexp" > gpurun_out/w8_probe.txt 2>&1
