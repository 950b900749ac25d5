#!/bin/bash
# rocprofv3 evidence for profiles/ (run on the GPU box): kernel traces of the
# timed steps of C2 / C3 / C4 / C5 (tools/kernel_stats.py) and PMC passes
# (tools/pmc_traffic.sh) -- kernel trace only, one counter group per pass.
# usage: tools/profile_configs.sh TAG [configs...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
NOX="--no-cpu-baseline --no-pcie --no-e2e --no-pipelined --no-match"
for cfg in "$@"; do
  case $cfg in
    c2) W=3; K=20; A="--config c2" ;;
    c3) W=1; K=3; A="--config c3" ;;
    c4) W=1; K=5; A="--config c4" ;;
    c5) W=1; K=5; A="--config c5" ;;
  esac
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$cfg -o run -- \
      python3 bench.py --steps $K --warmup $W $NOX $A > $O/trace_$cfg.log 2>&1 || exit $?
  python3 tools/kernel_stats.py $O/trace_$cfg $W $K $O/${cfg}_kernel_stats.csv || exit $?
  echo "$cfg trace done"
done
