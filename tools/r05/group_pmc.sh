#!/bin/bash
# C4 forward: event time and HBM fetch per causal head-group size variant (tools only)
L=$GRAFT_REPO_ROOT/hazyresearch_flash-attention_amd/flash_attn
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
bash tools/ab_libs.sh "C4" "fwd" "$@" > /dev/null 2>&1
grep event gpurun_out/ab_libs.txt
for t in prod "$@"; do
  if [ "$t" = prod ]; then unset FA_HIP_LIB; else export FA_HIP_LIB=$L/libfa_hip_$t.so; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/grp_pmc/$t -o p --output-format csv -- python tools/tiles_run.py --cfg C4 --mode fwd --launches 5 --warm 0.05 > /dev/null 2>&1
  echo "$t $(python tools/pmc_summary.py gpurun_out/grp_pmc/$t fa_fwd_d128 | tr -d '\n ')"
done
