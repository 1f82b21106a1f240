#!/bin/bash
# One config, several (library, impl) legs, one process each, interleaved, two rounds (tools only):
#   bash tools/r05/impl_ab.sh <cfg> "<lib:impl> ..."    (lib "prod" = the product libfa_hip.so)
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
for r in 1 2; do for leg in $2; do
  lib=${leg%%:*}; impl=${leg##*:}
  if [ "$lib" = prod ]; then
    timeout -k 10 120 python tools/tiles_run.py --cfg $1 --mode fwd --launches 200 --impl $impl 2>/dev/null | sed "s/^{/{\"lib\": \"prod\", /" || exit 1
  else
    FA_HIP_LIB=$L/libfa_hip_$lib.so timeout -k 10 120 python tools/tiles_run.py --cfg $1 --mode fwd --launches 200 --impl $impl 2>/dev/null | sed "s/^{/{\"lib\": \"$lib\", /" || exit 1
  fi
done; done
