#!/bin/bash
# Round-3 closing evidence in two gpurun calls (each under the 20-minute limit):
#   bash tools/round3_final.sh 1   bench (default and driver flags), rocprofv3 stats of the bench,
#                                  host cost, per-tile traces/PMC of D32 D64 D128
#   bash tools/round3_final.sh 2   per-tile traces/PMC of C2 C3 C4 C5
set -e
OUT=gpurun_out/r03f
mkdir -p $OUT
if [ "$1" = 1 ]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json.log 2>&1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extra > $OUT/bench_driver_flags.json.log 2>&1
  cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_bench -o b --output-format csv -- python bench.py --no-extra --no-cpu > $OUT/prof_bench.log 2>&1
  timeout -k 10 200 python -u tools/host_overhead.py > $OUT/host.json.log 2>&1
  bash tools/tiles_r03.sh $OUT/tiles D32 D64 D128
else
  bash tools/tiles_r03.sh $OUT/tiles C2 C3 C4 C5
fi
echo "part $1 done" > $OUT/DONE$1
