#!/bin/bash
# Round-4 first GPU batch: new robustness tests, PMC sweep of the north-star asm forward, per-workgroup
# timeline in real time and in shader cycles (loop cycles per tile).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_robustness.py tests/test_asm_forms.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k 'capture or churn or empty_key' > gpurun_out/t_r04a.txt 2>&1
echo "tests rc=$?" >> gpurun_out/t_r04a.txt
timeout -k 10 120 python -u tools/asm_wg_timeline.py > gpurun_out/wg_timeline_r04.txt 2>&1 || exit 1
timeout -k 10 120 python -u tools/asm_wg_timeline.py --cycles > gpurun_out/wg_timeline_r04_cyc.txt 2>&1 || exit 1
bash tools/pmc_sweep.sh gpurun_out/pmc_r04a --iters 10 && python tools/pmc_summary.py gpurun_out/pmc_r04a fa_fwd_d64p > gpurun_out/pmc_r04a.json
