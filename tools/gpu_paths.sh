# throughput of the other ordered paths on the C2 input
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-paths}
mkdir -p $O
B="--steps 5 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e --no-match --no-pipelined"
timeout -k 10 200 python -u bench.py $B --k 40 --prefix ATGAC > $O/k40.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B --k 70 --prefix ATGAC > $O/k70.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B --k 16 --prefix AT > $O/k16_AT.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B --k 21 --prefix "" --reads 4000000 > $O/k21_empty.log 2>&1 && \
timeout -k 10 200 python -u bench.py $B --k 16 --prefix ATGAC --flags 2 > $O/k16_records.log 2>&1
