#!/bin/bash
# Event-time A/B of library builds (tools only): the product libfa_hip.so and each
# flash_attn/libfa_hip_<tag>.so named on the command line, interleaved, two rounds.
#   bash tools/ab_libs.sh "<cfgs>" "<modes>" tag1 tag2 ...     -> gpurun_out/ab_libs.txt
set -e
CFGS=$1; MODES=$2; shift 2
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
for r in 1 2; do
for c in $CFGS; do for m in $MODES; do
  timeout -k 10 120 python tools/tiles_run.py --cfg $c --mode $m --launches 100 >> gpurun_out/ab_libs.txt 2>&1
  for t in "$@"; do
    FA_HIP_LIB=$L/libfa_hip_$t.so timeout -k 10 120 python tools/tiles_run.py --cfg $c --mode $m --launches 100 | sed "s/\"cfg\"/\"lib\": \"$t\", \"cfg\"/" >> gpurun_out/ab_libs.txt 2>&1
  done
done; done; done
