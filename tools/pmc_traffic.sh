#!/bin/bash
# HBM traffic of the bench kernels from PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a pass), kernel trace only -- no
# other trace domains.  Summarised by tools/pmc_traffic.py.
# usage: tools/pmc_traffic.sh TAG [bench args...]; then python tools/pmc_traffic.py gpurun_out/TAG CONFIG READS K PREFIX
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for c in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$OUT/pmc$i" -o run -- \
      python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie "$@" > "$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($c) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
