set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-quick}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie > gpurun_out/bench_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/prof_$TAG.log 2>&1
