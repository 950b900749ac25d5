#!/bin/bash
# narrow pass-1 keys (32 bits in B1, middle-base orientation for odd k): table tests, C5 pins, benches, A/B
set -o pipefail
O=gpurun_out/r06p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -k "fixed or canonical" > $O/pytest.txt 2>&1 || exit $?
bash tools/gpu_ab_env.sh r06p "--config c5 --steps 10 --warmup 2" ship "count:KMERHIP_TAB_P2=count" > $O/ab_c5.txt 2>&1 || exit $?
true
bash tools/pmc_traffic.sh r06p_pmc --config c5 --no-e2e --no-match --no-pipelined > $O/pmc.txt 2>&1 || exit $?
