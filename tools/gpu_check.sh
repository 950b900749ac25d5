#!/bin/bash
# One GPU call: the GPU test suite, then the C2 bench twice, then the
# two-rank rehearsal.  Stops at the first failing step.
# Output under gpurun_out/chk/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/chk
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-match --no-pcie"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/chk/pytest.txt 2>&1 || { tail -30 gpurun_out/chk/pytest.txt; exit 1; }
tail -2 gpurun_out/chk/pytest.txt
timeout -k 10 120 $B > gpurun_out/chk/c2_new.json 2> gpurun_out/chk/c2_new.err || { tail gpurun_out/chk/c2_new.err; exit 1; }
timeout -k 10 120 $B > gpurun_out/chk/c2_new2.json 2> gpurun_out/chk/c2_new2.err || { tail gpurun_out/chk/c2_new2.err; exit 1; }
python - <<'PY'
import json
for n in ("c2_new", "c2_new2"):
    d = json.load(open("gpurun_out/chk/%s.json" % n))
    print(n, "ms/step %.4f scan %.4f frac %.3f distinct %d" % (d["ms_per_step"], d["scan_kernel_ms"], d["roofline"]["frac"], d["distinct_kmers"]))
PY
[ "${SKIP_REH:-0}" = 1 ] || timeout -k 10 450 bash tools/rehearse_ranks.sh
