#!/bin/bash
# sort final with 16,384 bins for fixed regions (C3, C5): table tests, full-size pins, A/B
set -o pipefail
O=gpurun_out/r06t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_table_gpu.py tests/test_full_size_gpu.py -m gpu -q -x --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06t "--config c5 --steps 10 --warmup 2" ship "b8k:KMERHIP_TAB_BINS=8192" > $O/ab_c5.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06t_c3 "--config c3 --steps 3 --warmup 1" ship "b8k:KMERHIP_TAB_BINS=8192" > $O/ab_c3.txt 2>&1 || exit $?
