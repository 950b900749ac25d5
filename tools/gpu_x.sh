set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "exchange or sharded" > gpurun_out/pytest_x.log 2>&1 && \
timeout -k 10 200 python -u tools/exp_dist.py > gpurun_out/exp_dist.log 2>&1
