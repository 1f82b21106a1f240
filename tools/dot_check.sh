#!/bin/bash
# The backward pre-pass with every lane busy: GPU suite, then its kernel time per config (rocprofv3).
set -e
mkdir -p gpurun_out/dot
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_dot.txt 2>&1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for c in D32 D64 D128 C3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dot/$c -o t --output-format csv -- python tools/tiles_r03.py --cfg $c --mode bwd --launches 100 > gpurun_out/dot/$c.log 2>&1
done
