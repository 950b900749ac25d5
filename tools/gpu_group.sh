# group-context (ndev) tests through the C-ABI and readFile()
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-grp}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_node.py -m gpu -x -v --timeout 300 --timeout-method thread -k "group or node" > $O/pytest.log 2>&1
