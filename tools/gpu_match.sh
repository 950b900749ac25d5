set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-match}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_match_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
