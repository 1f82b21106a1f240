#!/bin/bash
# Round-4: price of the rescale test's dependence chain and of the per-block Q pre-scale.
mkdir -p gpurun_out
rm -f gpurun_out/pstamps_r04c.txt
for v in "" "--probe nobrdep" "--probe noqs" "--probe nobar,nobrdep"; do
  timeout -k 10 120 python -u tools/asm_pstamps.py --gen "$v" >> gpurun_out/pstamps_r04c.txt 2>&1 || exit 1
done
