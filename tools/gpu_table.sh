# table-mode tests (+ optional extra command), one GPU call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-table}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
