#!/bin/bash
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
bash tools/pmc_variant.sh gpurun_out/pmc_ps "--persist 1 --prescale 1 --kfirst 2 --xphase 1" && \
  python tools/pmc_summary.py gpurun_out/pmc_ps fa_fwd_d64p > gpurun_out/pmc_ps.json
bash tools/pmc_variant.sh gpurun_out/pmc_base "--persist 1" && \
  python tools/pmc_summary.py gpurun_out/pmc_base fa_fwd_d64p > gpurun_out/pmc_base.json
timeout -k 10 400 python -u tools/asm_variants.py --rounds 5 --variants \
  "pskx:--persist 1 --prescale 1 --kfirst 2 --xphase 1;pskxv2:--persist 1 --prescale 1 --kfirst 2 --xphase 1 --vp1 0;pskxl2:--persist 1 --prescale 1 --kfirst 2 --xphase 1 --lag 4,2;pskxl6:--persist 1 --prescale 1 --kfirst 2 --xphase 1 --lag 4,6" \
  > gpurun_out/var_r04c.txt 2>&1
