#!/bin/bash
# A/B of C2 bench runs: the shipping library ("ship") against other builds
# saved under kmerjs_amd/ (loaded through KMERHIP_LIB_EXPERIMENT), optionally
# with environment switches for the experiments build.
# usage: tools/gpu_ab.sh TAG ship|LIB[:VAR=val,...] ...
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; shift
mkdir -p gpurun_out/$TAG
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-match --no-pcie --no-pipelined"
i=0
for v in "$@"; do
  i=$((i+1))
  lib=${v%%:*}
  envs=""
  [ "$lib" != "$v" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
  n="$i-$(echo "$v" | tr '/:,=' '____')"
  if [ "$lib" = ship ]; then
    env $envs timeout -k 10 120 $B > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || { tail gpurun_out/$TAG/$n.err; exit 1; }
  else
    env KMERHIP_LIB_EXPERIMENT=kmerjs_amd/$lib $envs timeout -k 10 120 $B > gpurun_out/$TAG/$n.json 2> gpurun_out/$TAG/$n.err || { tail gpurun_out/$TAG/$n.err; exit 1; }
  fi
  python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/$n.json'))
print('$v', 'ms/step %.4f scan %.4f frac %.3f distinct %d' % (d['ms_per_step'], d['scan_kernel_ms'], d['roofline']['frac'], d['distinct_kmers']))"
done
