#!/bin/bash
# A/B of scan variants on C2 (experiments build, KMERHIP_SCAN=<variant>):
# usage: tools/gpu_ab.sh TAG variant...   ("ship" = the shipping library)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
mkdir -p gpurun_out/$TAG
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-match --no-pcie --no-pipelined"
for v in "$@"; do
  if [ "$v" = ship ]; then
    timeout -k 10 120 $B > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { tail gpurun_out/$TAG/$v.err; exit 1; }
  else
    KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so KMERHIP_SCAN=$v timeout -k 10 120 $B \
        > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { tail gpurun_out/$TAG/$v.err; exit 1; }
  fi
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/$TAG/$v.json'))
print('$v', 'ms/step %.4f scan %.4f frac %.3f distinct %d' % (d['ms_per_step'], d['scan_kernel_ms'], d['roofline']['frac'], d['distinct_kmers']))"
done
