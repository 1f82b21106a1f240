#!/bin/bash
# A/B of the backward / causal-forward block orders: the product library against one built with
# -DFA_BWD_XCD=0 (the round-2 orders) into flash_attn/libfa_hip_v0.so
#   FA_EXTRA_CFLAGS="-DFA_BWD_XCD=0" FA_BUILD_DIR=<dir> FA_BUILD_OUT=<repo>/hazyresearch_flash-attention_amd/flash_attn/libfa_hip_v0.so python hazyresearch_flash-attention_amd/build.py
#   bash tools/ab_xcd.sh "<cfgs>"     (event times -> gpurun_out/ab_xcd.txt, FETCH passes -> gpurun_out/ab_pmc/)
set -e
V0=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn/libfa_hip_v0.so
CFGS=${1:-C3 C4 D64}
for r in 1 2; do
for c in $CFGS; do for m in fwd bwd; do
  timeout -k 10 120 python tools/tiles_r03.py --cfg $c --mode $m --launches 100 >> gpurun_out/ab_xcd.txt 2>&1
  FA_HIP_LIB=$V0 timeout -k 10 120 python tools/tiles_r03.py --cfg $c --mode $m --launches 100 | sed 's/"cfg"/"lib": "v0", "cfg"/' >> gpurun_out/ab_xcd.txt 2>&1
done; done; done
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for c in $CFGS; do
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/ab_pmc/new_$c -o p --output-format csv -- python tools/tiles_r03.py --cfg $c --mode bwd --launches 5 --warm 0.05 > /dev/null 2>&1
done
