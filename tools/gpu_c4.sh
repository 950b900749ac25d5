# C4 pieces: exchange + device merge tests, the full-size C4 shard test,
# the C4 bench line, and a one-device two-rank rehearsal with --collect
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-c4}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread -k "exchange or c4_shard" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/c4.log 2>&1 && \
KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --reads 1000000 --steps 5 --warmup 1 --collect > $O/rehearse2.log 2>&1
