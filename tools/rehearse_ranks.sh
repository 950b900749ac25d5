#!/bin/bash
# Two ranks on ONE GPU over gloo: a rehearsal of the N > 1 bench paths (the
# driver runs the real multi-GPU scaling over RCCL on an 8-GPU node).  Uses
# bench.py's own launcher (`--gpus 2`, no torch.distributed.run), so the form
# the driver runs is the form rehearsed.  Every run verifies its result:
# C2 / C4 against the oracle on the whole job's input, C3 (table exchange) by
# the ranks' table digests and statistics adding up to one context's table.
# Output under gpurun_out/reh/ (the JSON lines say backend "gloo" and
# "REHEARSAL: every rank on device 0").
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/reh
export KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1
run() {   # name args...
  local n=$1; shift
  timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 1 "$@" \
      > gpurun_out/reh/$n.json 2> gpurun_out/reh/$n.err || { echo "$n failed"; tail -5 gpurun_out/reh/$n.err; exit 1; }
  grep -h "verify" gpurun_out/reh/$n.err > gpurun_out/reh/$n.verify.txt || { echo "$n: no verify line"; exit 1; }
  echo "$n ok: $(cat gpurun_out/reh/$n.verify.txt)"
}
run c2_hits --reads 1000000
run c4_dense --config c4 --reads 1000000
run c3_exchange --config c3 --reads 2000000
run c2_collect --collect --reads 1000000
