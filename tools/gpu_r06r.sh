#!/bin/bash
# no-prefix dense-hit path: count + write passes (shipping) vs every window ranked (round 5, KMERHIP_DENSE=slots)
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
bash tools/gpu_ab_env.sh r06r "--k 21 --prefix= --reads 4000000 --steps 5 --warmup 1 --no-cpu-baseline" ship "slots:KMERHIP_DENSE=slots" > $O/ab_k21.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06r_c5o "--config c5 --ordered --steps 5 --warmup 1" ship "slots:KMERHIP_DENSE=slots" > $O/ab_c5o.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06r_k16 "--prefix AT --steps 5 --warmup 1 --no-cpu-baseline" ship "slots:KMERHIP_DENSE=slots" > $O/ab_k16.txt 2>&1 || exit $?
