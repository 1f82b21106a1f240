#!/bin/bash
# Rotary kernel variants (tools only): the product and each flash_attn/libfa_hip_<tag>.so, two rounds
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
for r in 1 2; do
  echo "prod $(timeout -k 10 60 python tools/r05/rotary_time.py 2>/dev/null | grep rotary)"
  for t in "$@"; do echo "$t $(FA_HIP_LIB=$L/libfa_hip_$t.so timeout -k 10 60 python tools/r05/rotary_time.py 2>/dev/null | grep rotary)"; done
done
