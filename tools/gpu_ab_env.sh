#!/bin/bash
# A/B of experiment switches on one bench configuration:
# usage: tools/gpu_ab_env.sh TAG "bench args" variant...
#   variant = name (the shipping library) | name:VAR=val[,VAR=val] (the
#   experiments build with those KMERHIP_* variables)
set -o pipefail
cd "$(dirname "$0")/.."
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
B="python bench.py --no-cpu-baseline --no-e2e --no-match --no-pcie --no-pipelined $ARGS"
for v in "$@"; do
  name=${v%%:*}
  if [ "$name" = "$v" ]; then
    timeout -k 10 300 $B > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || { tail gpurun_out/$TAG/$name.err; exit 1; }
  else
    envs=$(echo "${v#*:}" | tr ',' ' ')
    env KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so $envs timeout -k 10 300 $B \
        > gpurun_out/$TAG/$name.json 2> gpurun_out/$TAG/$name.err || { tail gpurun_out/$TAG/$name.err; exit 1; }
  fi
  python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/$name.json'))
ph = d.get('table_phase_ms')
print('$name', 'ms/step %.4f kern %.4f frac %.3f distinct %d' % (d['ms_per_step'], d['scan_kernel_ms'], d['roofline']['frac'], d['distinct_kmers']), ' '.join('%s=%.2f' % kv for kv in (ph or {}).items()))"
done
