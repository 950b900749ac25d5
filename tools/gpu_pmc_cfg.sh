# kernel-trace stats + PMC traffic passes for the table-mode configs (c3, c5)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmccfg
mkdir -p $O
for c in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$c -o run -- \
      python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e > $O/stats_$c.log 2>&1 || exit $?
  echo "stats $c ok"
  timeout -k 10 600 bash tools/pmc_traffic.sh pmc_$c --config $c --no-e2e || exit $?
done
