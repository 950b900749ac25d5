#!/bin/bash
set -o pipefail
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 300 python -u tools/dense_debug.py > $O/dense_debug.jsonl 2> $O/dense_debug.err || exit $?
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_table_gpu.py tests/test_wide_keys_gpu.py tests/test_fasta_gpu.py "tests/test_full_size_gpu.py::test_c5_full_size_pins" -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -k 10 200 $B --prefix AT --steps 5 --warmup 1 > $O/k16_AT.json 2> $O/k16_AT.err || exit $?
timeout -k 10 200 $B --config c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err || exit $?
timeout -k 10 200 $B --config c5 --fasta --steps 10 --warmup 2 > $O/c5fa.json 2> $O/c5fa.err || exit $?
