#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
bash tools/tiles_r03.sh gpurun_out/r03d/tiles D128
