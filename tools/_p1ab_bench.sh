# C3 benches of the experiments build: fixed-run pass 1 at several run margins
# (KMERHIP_TAB_SIGMA) vs the counted pass (KMERHIP_TAB_P1=count)
set -o pipefail
mkdir -p gpurun_out/p1ab && export TMPDIR=/tmp
for v in fixed:1.5 fixed:2 fixed:2.5; do
  p=${v%%:*}; sg=${v#*:}; n=${p}_$sg
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_exp.so KMERHIP_TAB_SPILL_LOG=1 KMERHIP_TAB_P1=$p KMERHIP_TAB_SIGMA=$sg \
    timeout -k 10 300 python3 bench.py --config c3 --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/p1ab/$n.json 2> gpurun_out/p1ab/$n.err || { tail gpurun_out/p1ab/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/p1ab/$n.json')); print('$n', {k: d[k] for k in ('ms_per_step','value','unit')}); print(d.get('table_phase_ms'))"
  grep -m1 "tab pass 1" gpurun_out/p1ab/$n.err || true
done
