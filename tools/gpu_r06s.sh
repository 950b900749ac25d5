#!/bin/bash
# no-prefix dense hits back on the slots route: GPU tests of the ordered paths, benches
set -o pipefail
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_keys_gpu.py tests/test_full_size_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -k 10 200 $B --k 21 --prefix= --reads 4000000 --steps 5 --warmup 1 > $O/k21.json 2> $O/k21.err || exit $?
timeout -k 10 200 $B --config c5 --ordered --steps 5 --warmup 1 > $O/c5o.json 2> $O/c5o.err || exit $?
