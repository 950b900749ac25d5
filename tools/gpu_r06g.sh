#!/bin/bash
# C5 / C5 FASTA: wave final (shipping) vs the counted pass 2 + sort final (experiments build), same box
set -o pipefail
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_table_gpu.py "tests/test_full_size_gpu.py::test_c5_full_size_pins" -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06g "--config c5 --steps 10 --warmup 2" wave "count:KMERHIP_TAB_P2=count" > $O/ab_c5.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06g_fa "--config c5 --fasta --steps 10 --warmup 2" wave "count:KMERHIP_TAB_P2=count" > $O/ab_c5fa.txt 2>&1 || exit $?
