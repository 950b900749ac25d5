#!/bin/bash
# round 6: bucket_scatter race probe (three builds) + the GPU suite on the shipping build
set -o pipefail
mkdir -p gpurun_out/r06a
for b in nofix fix; do
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_probe_$b.so timeout -k 10 180 python -u tools/bkt_race_probe.py $b 3 >> gpurun_out/r06a/probe.jsonl 2>> gpurun_out/r06a/probe.err || exit $?
done
timeout -k 10 180 python -u tools/bkt_race_probe.py shipping 3 >> gpurun_out/r06a/probe.jsonl 2>> gpurun_out/r06a/probe.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06a/pytest_gpu.txt 2>&1
