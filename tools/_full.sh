mkdir -p gpurun_out/full && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_sessions_gpu.py tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/full/pytest.txt 2>&1 || { tail -30 gpurun_out/full/pytest.txt; exit 1; }
tail -1 gpurun_out/full/pytest.txt
