# C2 bench under KMER_FLAG_ABLATE_* flag values (experiments; results are not counts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
for f in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-pcie --steps 10 --flags $f > gpurun_out/ab_${TAG}_f$f.log 2>&1 || exit $?
done
