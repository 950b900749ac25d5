#!/bin/bash
set -o pipefail
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 300 python -u tools/dense_debug.py > $O/dense_debug.jsonl 2> $O/dense_debug.err || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_keys_gpu.py tests/test_step_gpu.py tests/test_long_lines_gpu.py tests/test_table_gpu.py tests/test_general_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
B="python bench.py --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -k 10 200 $B --prefix AT --steps 5 --warmup 1 > $O/k16_AT.json 2> $O/k16_AT.err || exit $?
timeout -k 10 200 $B --k 64 --prefix AT --reads 2000000 --steps 3 --warmup 1 > $O/k64_AT.json 2> $O/k64_AT.err || exit $?
timeout -k 10 200 $B --steps 20 --warmup 3 > $O/c2.json 2> $O/c2.err || exit $?
timeout -k 10 300 $B --config c3 --steps 3 --warmup 1 > $O/c3.json 2> $O/c3.err || exit $?
