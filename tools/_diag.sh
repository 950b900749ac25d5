# ordered k=3 parity under stale / poisoned device memory, then the C3 pass-1 A/B
set -o pipefail
mkdir -p gpurun_out/diag && export TMPDIR=/tmp
T="python -u -m pytest -q --timeout 200 --timeout-method thread"
timeout -k 10 300 $T tests/test_table_gpu.py -k "line_split" > gpurun_out/diag/ship_ls.log 2>&1; echo "ship line_split rc=$?"; tail -3 gpurun_out/diag/ship_ls.log
KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so KMERHIP_POISON=1 timeout -k 10 400 $T tests/test_table_gpu.py tests/test_gpu_parity.py > gpurun_out/diag/poison.log 2>&1; echo "poison rc=$?"; grep -E "^FAILED|passed|failed" gpurun_out/diag/poison.log | head -20
STEPS=3 bash tools/_p1ab_bench.sh
