#!/bin/bash
# round 6: race probe (longer delay) + dense-path parity + dense benches
set -o pipefail
O=gpurun_out/r06b
mkdir -p $O
for b in fix; do
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_probe_$b.so timeout -k 10 300 python -u tools/bkt_race_probe.py $b 2 >> $O/probe.jsonl 2>> $O/probe.err || exit $?
done
timeout -k 10 300 python -u tools/bkt_race_probe.py shipping 2 >> $O/probe.jsonl 2>> $O/probe.err || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_keys_gpu.py tests/test_step_gpu.py tests/test_long_lines_gpu.py tests/test_table_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_dense.txt 2>&1 || exit $?
for cfg in "k16_AT --prefix AT --steps 5 --warmup 1" "k16_ACG --prefix ACG --steps 5 --warmup 1" "k64_AT --k 64 --prefix AT --reads 2000000 --steps 3 --warmup 1" "k21_noprefix --k 21 --prefix '' --reads 4000000 --steps 5 --warmup 1" "c5_ordered --config c5 --ordered --steps 5 --warmup 1" "c2 --steps 20 --warmup 3"; do
  set -- $cfg; name=$1; shift
  eval timeout -k 10 400 python bench.py "$@" --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > $O/$name.log 2>&1 || exit $?
  grep '^{' $O/$name.log > $O/$name.json || true
done
