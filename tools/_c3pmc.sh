# C3 HBM traffic per kernel (FETCH_SIZE / WRITE_SIZE in separate passes), one timed step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c3pmc
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc1 -o run -- python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc1.log 2>&1 && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc2 -o run -- python3 bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc2.log 2>&1
