set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-c3c5t}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_table_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-e2e > $O/c3.log 2>&1
