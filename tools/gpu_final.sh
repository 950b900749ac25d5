# Round-end evidence: full GPU suite, default bench line, C2 kernel stats,
# C3 PMC traffic passes (the final kernel changed).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-e2e > $O/prof.log 2>&1 && \
bash tools/pmc_traffic.sh ${1:-final}_pmc_c3 --config c3 --no-e2e
