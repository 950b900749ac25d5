#!/bin/bash
# One gpurun session: GPU tests, bench, rocprofv3 kernel trace.  Each GPU step
# has its own time limit; a fault/abort/timeout (rc not in {0,1}) ends the run.
# usage: tools/gpu_check.sh [tag] [pytest-args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r01}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
rc_ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }

echo "== pytest -m gpu" | tee "$OUT/steps.log"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout=600 "$@" > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a "$OUT/steps.log"; tail -30 "$OUT/pytest_gpu.log"
rc_ok $rc || exit $rc

echo "== smoke" | tee -a "$OUT/steps.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc" | tee -a "$OUT/steps.log"; tail -5 "$OUT/smoke.log"
rc_ok $rc || exit $rc

echo "== bench" | tee -a "$OUT/steps.log"
timeout -k 10 600 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc" | tee -a "$OUT/steps.log"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
rc_ok $rc || exit $rc

echo "== rocprofv3 kernel trace" | tee -a "$OUT/steps.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc" | tee -a "$OUT/steps.log"
find "$OUT/prof" -name "*stats*" | head
exit 0
