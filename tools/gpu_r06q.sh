#!/bin/bash
# after narrow pass-1 keys: full GPU suite, C5 / C5 FASTA profiles, C3 bench line
set -o pipefail
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || exit $?
bash tools/profile_configs.sh r06q c5 c5fa || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > $O/c3.json 2> $O/c3.err || exit $?
