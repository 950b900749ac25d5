set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-long}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_long_lines_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
