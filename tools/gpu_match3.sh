set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-match3}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_match_gpu.py tests/test_node.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_match.py > $O/bench_match.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u tools/bench_match.py --no-cpu-baseline --steps 2 > $O/prof.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-e2e > $O/c3.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_table_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_table.log 2>&1
