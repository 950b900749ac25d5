#!/bin/bash
# the no-prefix dense-hit lines again with the corrected roofline label
set -o pipefail
O=gpurun_out/r06f_rb
mkdir -p $O
timeout -k 10 400 python bench.py --config c5 --ordered --steps 10 --warmup 2 > $O/c5_ordered.log 2>&1 || exit $?
grep '^{' $O/c5_ordered.log > $O/c5_ordered.json || exit $?
timeout -k 10 400 python bench.py --k 21 --prefix "" --reads 4000000 --steps 5 --warmup 1 --no-cpu-baseline > $O/k21_noprefix.log 2>&1 || exit $?
grep '^{' $O/k21_noprefix.log > $O/k21_noprefix.json || exit $?
