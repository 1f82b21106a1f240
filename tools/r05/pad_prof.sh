#!/bin/bash
# rocprofv3 kernel times of the var-len gather / scatter (tools only)
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/r05/pad_time.py
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/padprof -o r --output-format csv -- python tools/r05/pad_time.py > /dev/null 2>&1
cat $(ls gpurun_out/padprof/*/r_kernel_stats.csv 2>/dev/null || ls gpurun_out/padprof/r_kernel_stats.csv) | cut -d, -f1-4 | head -8
