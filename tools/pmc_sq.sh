#!/bin/bash
# One PMC pass of SQ instruction counters over a short bench run (kernel trace only).
set -u
cd "$(dirname "$0")/.."
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SMEM \
    --kernel-trace --output-format csv -d "$OUT/pmc1" -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie "$@" > "$OUT/pmc1.log" 2>&1
