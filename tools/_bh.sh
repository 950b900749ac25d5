export TMPDIR=/tmp; mkdir -p gpurun_out/bh
KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_bh2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/bh/pytest2.txt 2>&1 || { tail -20 gpurun_out/bh/pytest2.txt; exit 1; }
KMERHIP_LIB_EXPERIMENT=kmerjs_amd/libkmerhip_bh4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/bh/pytest4.txt 2>&1 || { tail -20 gpurun_out/bh/pytest4.txt; exit 1; }
tail -1 gpurun_out/bh/pytest2.txt; tail -1 gpurun_out/bh/pytest4.txt
for lib in libkmerhip.so libkmerhip_bh2.so libkmerhip_bh4.so; do
timeout -k 10 200 env KMERHIP_LIB_EXPERIMENT=kmerjs_amd/$lib rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bh/$lib -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-match --no-pcie --no-pipelined > gpurun_out/bh/$lib.json 2> gpurun_out/bh/$lib.err || { tail gpurun_out/bh/$lib.err; exit 1; }
f=$(find gpurun_out/bh/$lib -name "*kernel_stats.csv" | head -1); echo $lib $(grep bucket_heads $f | cut -d, -f4) $(python3 -c "import json; d=json.load(open('gpurun_out/bh/$lib.json')); print(d['ms_per_step'], d['distinct_kmers'])")
done
