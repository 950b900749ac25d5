set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cfg}
for c in c3 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$c -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$c.log 2>&1 || exit $?
done
