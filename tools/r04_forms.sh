#!/bin/bash
# Round-4: forward forms per configuration (event time, tools/tiles_run.py --impl).
mkdir -p gpurun_out
rm -f gpurun_out/forms_r04.txt
for c in C2 C5 C3nd; do for i in auto asm4 asm4p hip; do   # (asm8: left the library in round 6)
  timeout -k 10 120 python tools/tiles_run.py --cfg $c --mode fwd --impl $i --launches 100 >> gpurun_out/forms_r04.txt 2>&1 || exit 1
done; done
