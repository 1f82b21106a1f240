#!/bin/bash
# rocprofv3 kernel times of the rotary kernel variants (tools only)
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
for t in prod "$@"; do
  if [ "$t" = prod ]; then unset FA_HIP_LIB; else export FA_HIP_LIB=$L/libfa_hip_$t.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/rotprof/$t -o r --output-format csv -- python tools/r05/rotary_time.py > /dev/null 2>&1
  f=$(ls gpurun_out/rotprof/$t/*/r_kernel_stats.csv 2>/dev/null || ls gpurun_out/rotprof/$t/r_kernel_stats.csv)
  echo "$t $(grep rotary $f | cut -d, -f1-4)"
done
