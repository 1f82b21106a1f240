#!/bin/bash
# Forward forms at the north star and neighbours, one process per (cfg, impl), interleaved, two rounds:
#   bash tools/r05/forms_ab.sh "<cfgs>" "<impls>" > gpurun_out/<out>.txt
for r in 1 2; do
for c in $1; do for i in $2; do
  timeout -k 10 120 python tools/tiles_run.py --cfg $c --mode fwd --launches 200 --impl $i 2>/dev/null || exit 1
done; done; done
