set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-e2e --no-match > gpurun_out/$TAG.log 2>&1
