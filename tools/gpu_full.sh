set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > gpurun_out/$TAG.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_dist.py > gpurun_out/exp_dist.log 2>&1
