#!/bin/bash
# Round-end evidence: GPU tests, smoke, the default bench line, the rocprofv3 kernel-trace/stats
# summary of the same bench command, kernel traces of the other BASELINE configs (C2..C5, fwd and
# fwd+bwd), and the forward's HBM bytes / MFMA busy from separate PMC passes.
#   bash tools/round_end_profile.sh <tag> [skip-tests]     (outputs under gpurun_out/<tag>/)
set -e
TAG=${1:-rXX}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
fi
timeout -k 10 600 python bench.py > "$OUT/bench.json.log" 2>&1
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_bench" -o b --output-format csv -- python bench.py --no-extra --no-cpu > "$OUT/prof_bench.log" 2>&1
# kernel traces of the other configs: C2 fwd, C3 fwd+bwd (causal, dropout), C4 fwd+bwd (D=128 causal), C5 fwd
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c2" -o k --output-format csv -- python tools/run_fwd.py --B 8 --H 12 --S 512 --D 64 --fp16 1 --iters 50 > "$OUT/prof_c2.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c3" -o k --output-format csv -- python tools/run_fwd.py --B 8 --H 12 --S 2048 --D 64 --causal 1 --p 0.1 --bwd 1 --iters 30 > "$OUT/prof_c3.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o k --output-format csv -- python tools/run_fwd.py --B 16 --H 12 --S 4096 --D 128 --causal 1 --bwd 1 --iters 10 > "$OUT/prof_c4.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o k --output-format csv -- python tools/run_fwd.py --B 4 --H 16 --S 1024 --Sk 4096 --D 64 --iters 50 > "$OUT/prof_c5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU -d "$OUT/pmc_mfma" -o p --output-format csv -- python tools/run_fwd.py --iters 5 > "$OUT/pmc_mfma.log" 2>&1
echo done > "$OUT/DONE"
