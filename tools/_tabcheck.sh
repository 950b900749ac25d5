# table-mode checks after a pass-1 change: table tests, C3 full-size properties, C3 and C5 benches
set -o pipefail
mkdir -p gpurun_out/tabcheck && export TMPDIR=/tmp
O=gpurun_out/tabcheck
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_table_gpu.py "tests/test_full_size_gpu.py::test_c3_full_size_properties" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for cfg in c3 c5; do
  timeout -k 10 300 python3 bench.py --config $cfg --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || { tail $O/$cfg.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$cfg.json')); print('$cfg', {k: d[k] for k in ('ms_per_step','value')}, d.get('table_phase_ms'))"
done
