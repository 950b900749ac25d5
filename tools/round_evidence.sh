#!/bin/bash
# Round-end evidence on one GPU: the GPU test suite, smoke() and the default
# bench line (gpurun_out/TAG/); each step under its own time limit, stopping
# at the first failure.  usage: tools/round_evidence.sh TAG
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest rc=$?"; exit 1; }
tail -3 "$OUT/pytest_gpu.txt"
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$OUT/smoke.txt" 2>&1 || { echo "smoke rc=$?"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench_default.log" 2>&1 || { echo "bench rc=$?"; exit 1; }
grep '^{' "$OUT/bench_default.log" > "$OUT/bench_default.json" || true
cat "$OUT/bench_default.json"
