mkdir -p gpurun_out/$CFG && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$CFG/p -o run -- python3 bench.py --config $CFG --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/$CFG/b.json 2> gpurun_out/$CFG/b.err || { tail gpurun_out/$CFG/b.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/$CFG/b.json')); print({k: d[k] for k in ('ms_per_step','value','unit')}); print(d.get('phases_ms') or d.get('phase_ms'))"
f=$(find gpurun_out/$CFG/p -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -16
