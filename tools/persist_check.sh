#!/bin/bash
# GPU check of the persistent asm forward in the product path: the form tests first, then the whole
# -m gpu suite, then the bench (north star through the interface).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_asm_forms.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_forms.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_persist.txt 2>&1
timeout -k 10 300 python -u bench.py --no-extra > gpurun_out/bench_persist.json.log 2>&1
