#!/bin/bash
# Final GPU check of the build: asm form tests, the whole -m gpu suite, smoke(), bench.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_asm_forms.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_forms2.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_final.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.txt 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_final.json.log 2>&1
