mkdir -p gpurun_out/swz2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_gpu.py tests/test_wide_keys_gpu.py tests/test_step_gpu.py tests/test_fasta_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/swz2/pytest.txt 2>&1 || { tail -30 gpurun_out/swz2/pytest.txt; exit 1; }
tail -1 gpurun_out/swz2/pytest.txt
B="python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-match --no-pcie --no-pipelined"
run() { n=$1; lib=$2
  env KMERHIP_LIB_EXPERIMENT=kmerjs_amd/$lib timeout -k 10 120 $B > gpurun_out/swz2/$n.json 2> gpurun_out/swz2/$n.err || { tail gpurun_out/swz2/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/swz2/$n.json'))
print('$n', 'ms/step %.4f scan %.4f frac %.3f distinct %d' % (d['ms_per_step'], d['scan_kernel_ms'], d['roofline']['frac'], d['distinct_kmers']))"
}
run swz1 libkmerhip.so && run noswz1 libkmerhip_noswz.so && run swz2 libkmerhip.so && run noswz2 libkmerhip_noswz.so || exit 1
for lib in libkmerhip.so libkmerhip_noswz.so; do
  KMERHIP_LIB_EXPERIMENT=kmerjs_amd/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/swz2/pmc_$lib -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined > gpurun_out/swz2/pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 gpurun_out/swz2/pmc_$lib.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for lib in ("libkmerhip.so", "libkmerhip_noswz.so"):
    agg = collections.defaultdict(list)
    for f in glob.glob("gpurun_out/swz2/pmc_%s/**/*counter_collection.csv" % lib, recursive=True):
        for r in csv.DictReader(open(f)):
            if "scan_planes" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(lib, {k: "%.4g" % (sum(v) / len(v)) for k, v in sorted(agg.items())})
PY
