# Re-verify the tree: GPU suite, default bench line, C3 (kernel stats) and C5 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-verify3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e > $O/c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1
