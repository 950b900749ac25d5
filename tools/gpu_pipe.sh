# sequential vs pipelined bench (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pipe}
for n in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --pipeline $n > gpurun_out/ab_${TAG}_p$n.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --pipeline 3 > gpurun_out/prof_$TAG.log 2>&1
