#!/bin/bash
# table mode: the capacity check deferred past the finals, one wait less after pass 1; tests, C5 / C5 FASTA / C3 lines
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_table_gpu.py "tests/test_full_size_gpu.py::test_c5_full_size_pins" -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
B="python bench.py --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -k 10 200 $B --config c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err || exit $?
timeout -k 10 200 $B --config c5 --fasta --steps 10 --warmup 2 > $O/c5fa.json 2> $O/c5fa.err || exit $?
timeout -k 10 300 $B --config c3 --steps 3 --warmup 1 > $O/c3.json 2> $O/c3.err || exit $?
