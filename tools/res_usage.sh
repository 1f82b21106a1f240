#!/bin/bash
# Print register / spill usage of the forward kernels of one head-dim TU under extra -D flags.
#   tools/res_usage.sh <d32|d64|d128>_<fwd|bwd> [kernel-substring] [-DFOO=1 ...]
# (build.py SOURCE_FLAGS are not applied: pass them as extra flags)
TU=$1; shift
MFMAFORM=${MFMAFORM--mllvm -amdgpu-mfma-vgpr-form}
PAT=${1:-fa_fwd_kernel}; shift
cd "$(dirname "$0")/../hazyresearch_flash-attention_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -I ../include -I csrc $MFMAFORM \
  --cuda-device-only -S -x hip csrc/fa_$TU.hip  -o /tmp/fa_$TU.s -Rpass-analysis=kernel-resource-usage "$@" 2>&1 |
  grep -A12 "Function Name: .*$PAT" | grep -E "Function Name|VGPRs:|AGPRs|Spill|Occupancy" |
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - - - 
