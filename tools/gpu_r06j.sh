#!/bin/bash
# table mode: pass 2 into narrow 32-bit keys in fixed regions (k <= 21) -- tests, then A/B against the counted pass 2
set -o pipefail
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_table_gpu.py tests/test_fasta_gpu.py "tests/test_full_size_gpu.py::test_c5_full_size_pins" -m gpu -v -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06j "--config c5 --steps 10 --warmup 2" ship "old:KMERHIP_TAB_P2=count" > $O/ab_c5.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06j_fa "--config c5 --fasta --steps 10 --warmup 2" ship "old:KMERHIP_TAB_P2=count" > $O/ab_c5fa.txt 2>&1 || exit $?
