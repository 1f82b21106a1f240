#!/bin/bash
# Round-end evidence: GPU tests, smoke, the default bench line, the rocprofv3 kernel-trace/stats
# summary of the same bench command, and the forward's HBM bytes from separate PMC passes.
#   bash tools/round_end_profile.sh <tag>      (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -x -q -m "gpu and not slow" > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 600 python bench.py > "$OUT/bench.json.log" 2>&1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o b --output-format csv -- python bench.py --no-extra --no-cpu > "$OUT/prof_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU -d "$OUT/pmc_mfma" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_mfma.log" 2>&1
echo done > "$OUT/DONE"
