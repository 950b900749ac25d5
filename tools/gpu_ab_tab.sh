# A/B of table-kernel variants ab/<v>.so on C5 and C3 (first variant's table
# parity tests run first)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
first=1
for v in "$@"; do
  cp ab/$v.so kmerjs_amd/libkmerhip.so || exit 1
  if [ $first = 1 ]; then
    timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/abt_${TAG}_${v}_pytest.log 2>&1 || exit $?
    first=0
  fi
  timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > gpurun_out/abt_${TAG}_${v}_c5.log 2>&1 && \
  timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-e2e > gpurun_out/abt_${TAG}_${v}_c3.log 2>&1 || exit $?
done
