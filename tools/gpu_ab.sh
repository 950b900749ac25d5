# A/B: the in-tree library vs exp/<variant>.so on a bench config (no tests);
# extra bench arguments in $BENCH_ARGS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie $BENCH_ARGS > gpurun_out/ab_${TAG}_base.log 2>&1 || exit $?
for v in "$@"; do
  cp exp/$v.so kmerjs_amd/libkmerhip.so && \
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie $BENCH_ARGS > gpurun_out/ab_${TAG}_$v.log 2>&1 || exit $?
done
