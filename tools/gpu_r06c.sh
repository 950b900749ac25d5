#!/bin/bash
set -o pipefail
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 400 python -u tools/dense_debug.py > $O/dense_debug.jsonl 2> $O/dense_debug.err || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_keys_gpu.py tests/test_step_gpu.py tests/test_long_lines_gpu.py tests/test_table_gpu.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_dense.txt 2>&1
exit 0
