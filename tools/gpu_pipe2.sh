set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe2}
mkdir -p $O
for p in 1 2 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-pcie --no-e2e --no-match --pipeline $p > $O/p$p.$RANDOM.log 2>&1 || exit $?
done
