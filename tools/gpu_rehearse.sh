set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --reads 1000000 --steps 5 --warmup 1 > gpurun_out/rehearse2.log 2>&1 && \
KMERHIP_ONE_DEVICE=1 KMERHIP_DIST_BACKEND=gloo KMERHIP_BENCH_VERIFY=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 3 --reads 300000 --steps 3 --warmup 1 --k 13 --prefix AC > gpurun_out/rehearse3.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
