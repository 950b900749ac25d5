set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tabprof}
mkdir -p $O
export KMERHIP_LIB_EXPERIMENT=abtest/libkmerhip_prof.so KMERHIP_TAB_PROF=1
timeout -k 10 200 python -u bench.py --config c5 --steps 2 --warmup 0 --no-cpu-baseline --no-pcie > $O/c5.log 2>&1 && \
KMERHIP_TAB_RANGE=100000 timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-pcie > $O/c5_r1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c3 --steps 1 --warmup 0 --no-cpu-baseline --no-pcie --no-e2e > $O/c3.log 2>&1
