set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-canon}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --ordered --prefix ATGAC --steps 5 --warmup 1 > $O/c5o.log 2>&1
