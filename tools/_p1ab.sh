# C3 pass-1 A/B: table GPU tests, then C3 benches of the experiments build
# with the fixed-run pass 1 (default) and the counted one (KMERHIP_TAB_P1=count)
set -o pipefail
mkdir -p gpurun_out/p1ab && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_table_gpu.py > gpurun_out/p1ab/t.log 2>&1 || { tail -30 gpurun_out/p1ab/t.log; exit 1; }
tail -2 gpurun_out/p1ab/t.log
for v in fixed count; do
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so KMERHIP_TAB_SPILL_LOG=1 KMERHIP_TAB_P1=$v \
    timeout -k 10 300 python3 bench.py --config c3 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/p1ab/$v.json 2> gpurun_out/p1ab/$v.err || { tail gpurun_out/p1ab/$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/p1ab/$v.json')); print('$v', {k: d[k] for k in ('ms_per_step','value','unit')}); print(d.get('phases_ms') or d.get('phase_ms'))"
  grep -m3 "tab pass 1" gpurun_out/p1ab/$v.err || true
done
