#!/bin/bash
# Evidence for the persistent forward in the product: bench (default and driver flags), rocprofv3
# stats of the bench command, per-tile traces/PMC of D64 (the config whose kernel changed).
set -e
OUT=gpurun_out/r03p
mkdir -p $OUT
timeout -k 10 400 python -u bench.py > $OUT/bench.json.log 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra > $OUT/bench_driver_flags.json.log 2>&1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o b --output-format csv -- python bench.py --no-extra --no-cpu > $OUT/prof_bench.log 2>&1
bash tools/tiles_r03.sh $OUT/tiles D64
echo done > $OUT/DONE
