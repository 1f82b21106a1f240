#!/bin/bash
# Round-6 closing evidence (tools only): the round-end profile of the shipped build (GPU tests, smoke,
# bench line, rocprofv3 stats of the bench command and of C2..C5, forward PMC), then the forward's PMC
# issue/co-execution counters for the shipped library and the round-5-equivalent variant library
# (libfa_hip_r5eq.so: gen_fwd.py --soff 0 --carry 0 --proorder 0), then the per-block stamp anatomy.
#   bash tools/r06_round_end.sh <tag>
set -e
TAG=${1:-r06}
bash tools/round_end_profile.sh "$TAG"
bash tools/r05/forms_pmc.sh "$GRAFT_REPO_ROOT/gpurun_out/$TAG/forms_pmc" "prod:asm4p r5eq:asm4p"
timeout -k 10 300 python tools/asm_pstamps.py > "gpurun_out/$TAG/pstamps.txt" 2>&1
echo done > "gpurun_out/$TAG/DONE2"
