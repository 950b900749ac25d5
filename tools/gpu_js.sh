# Node drop-in tests, gzip/writer parity, and the C2 bench line (with the
# end-to-end readFile() run and the threaded CPU baseline), one GPU call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-js}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_node.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "node or gzip" > $O/pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1
