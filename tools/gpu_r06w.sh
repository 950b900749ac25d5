#!/bin/bash
# sanity after reverting the deferred verification: ordered-path tests, default bench
set -o pipefail
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py::test_c2_full_size_properties -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit $?
