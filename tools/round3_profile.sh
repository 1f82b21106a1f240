#!/bin/bash
# Round-3 end-of-round evidence (outputs under gpurun_out/r03/): bench line (default flags and the
# driver's), rocprofv3 kernel-trace/stats of the bench command, host cost per call.
set -e
OUT=gpurun_out/r03
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra > $OUT/bench_driver_flags.json.log 2>&1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o b --output-format csv -- python bench.py --no-extra --no-cpu > $OUT/prof_bench.log 2>&1
timeout -k 10 200 python -u tools/host_overhead.py > $OUT/host.json.log 2>&1
echo done > $OUT/DONE
