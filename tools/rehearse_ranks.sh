#!/bin/bash
# Two ranks on ONE GPU with gloo (rehearsal of the N > 1 bench paths; the
# driver runs the real multi-GPU scaling with RCCL): C2 hit exchange with the
# oracle check, C4 dense reduce-scatter merge, C3 table key exchange, C2 with
# the device collect.  Output under gpurun_out/reh/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/reh
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
export KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1
run() {   # name port args...
  local n=$1 p=$2; shift 2
  timeout -k 10 240 $R --master-port $p bench.py --gpus 2 --steps 3 --warmup 1 "$@" \
      > gpurun_out/reh/$n.json 2> gpurun_out/reh/$n.err || { echo "$n failed"; tail -5 gpurun_out/reh/$n.err; exit 1; }
  echo "$n ok"
}
run c2_hits 29611 --reads 1000000
run c4_dense 29612 --config c4 --reads 1000000
run c3_exchange 29613 --config c3 --reads 2000000
run c2_collect 29614 --collect --reads 1000000
grep -h "verify" gpurun_out/reh/*.err
