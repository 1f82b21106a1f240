#!/bin/bash
# Round-4 product check: the whole -m gpu suite (all failures listed), smoke(), the default bench line,
# then (if time allows) the backward no-atomics probe A/B and PMC of the product forward.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/gputest_r04.txt 2>&1
echo "suite rc=$?" >> gpurun_out/gputest_r04.txt
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-extra > gpurun_out/bench_r04.json 2>&1 || exit 1
rm -f gpurun_out/ab_libs.txt
timeout -k 10 200 bash tools/ab_libs.sh "D64 C3" "bwd" noat || exit 1
bash tools/pmc_sweep.sh gpurun_out/pmc_r04p --iters 10 && python tools/pmc_summary.py gpurun_out/pmc_r04p fa_fwd_d64p > gpurun_out/pmc_r04p.json
