# C3 (table mode, 100 M reads) and C4 (125 M reads per GPU) bench lines + a
# kernel-trace profile of C3, one GPU call
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-big}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > $O/c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/c4.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --config c3 --steps 2 --warmup 1 > $O/prof_c3.log 2>&1
