# Table mode: parity (incl. the multi-rank exchange), C3 / C5 bench lines,
# C3 kernel stats, and a two-rank C3 rehearsal on one device (gloo).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-tabx}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_table_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-pcie --no-e2e > $O/c3.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 1 > $O/c5.log 2>&1 && \
KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --config c3 --reads 4000000 --steps 3 --warmup 1 --no-e2e > $O/c3_rehearse2.log 2>&1
