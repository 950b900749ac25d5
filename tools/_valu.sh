mkdir -p gpurun_out/valu && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_wide_keys_gpu.py tests/test_step_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/valu/pytest.txt 2>&1 || { tail -30 gpurun_out/valu/pytest.txt; exit 1; }
tail -1 gpurun_out/valu/pytest.txt
bash tools/gpu_ab.sh valu ship libkmerhip_base.so ship libkmerhip_base.so || exit 1
for lib in libkmerhip.so libkmerhip_base.so; do
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/valu/pmc_$lib -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > gpurun_out/valu/pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 gpurun_out/valu/pmc_$lib.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for lib in ("libkmerhip.so", "libkmerhip_base.so"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/valu/pmc_%s/**/*counter_collection.csv" % lib, recursive=True):
        for r in csv.DictReader(open(f)):
            if "scan_planes" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(lib, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
