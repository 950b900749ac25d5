#!/bin/bash
# C5 pass 1: formation alone (the counted pass's tab_hist1) vs the fixed-run scatter
set -o pipefail
O=gpurun_out/r06o
mkdir -p $O
bash tools/gpu_ab_env.sh r06o "--config c5 --steps 10 --warmup 2" ship "count:KMERHIP_TAB_P1=count" > $O/ab_c5.txt 2>&1 || exit $?
