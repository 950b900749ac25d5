#!/bin/bash
# deferred verification of the scan's candidates (verify_kernel): ordered-path GPU tests, C2 A/B
set -o pipefail
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py::test_c2_full_size_properties tests/test_sessions_gpu.py tests/test_long_lines_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06u "--steps 20 --warmup 3" ship "old:KMERHIP_SCAN_DV=0" > $O/ab_c2.txt 2>&1 || exit $?
bash tools/gpu_r06v.sh || exit $?
