#!/bin/bash
# C5: the cost of pass 1's key mix (experiments build, KMERHIP_TAB_HASH=shift: a rotation, results wrong)
set -o pipefail
O=gpurun_out/r06l
mkdir -p $O
bash tools/gpu_ab_env.sh r06l "--config c5 --steps 10 --warmup 2" ship "shift:KMERHIP_TAB_HASH=shift" > $O/ab_c5.txt 2>&1 || exit $?
