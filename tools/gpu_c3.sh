# table-mode tests + C3 bench line, one GPU call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-c3}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > $O/c3.log 2>&1
